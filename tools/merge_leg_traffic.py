#!/usr/bin/env python3
"""Replace one leg of a traffic record with a fresh tools/pmc_traffic.py output:
   merge_leg_traffic.py <record.json> <new.json> <leg>"""
import json, sys
rec, new, leg = sys.argv[1:4]
r = json.load(open(rec))
r["legs"][leg] = json.load(open(new))["legs"][leg]
json.dump(r, open(rec, "w"), indent=1)
print(leg, r["legs"][leg]["traffic_bytes"])
