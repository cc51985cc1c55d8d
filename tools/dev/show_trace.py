#!/usr/bin/env python3
"""Dev: print a decode_trace.py JSON (one layer) as a table."""
import json
import sys

txt = open(sys.argv[1]).read()
d = json.loads(txt[txt.index("{"):])
print(d["step_us"], d["per_layer_us"], d["status"])
for k in sys.argv[2:] or ["layer4"]:
    for e, v in d[k].items():
        print(f"{e:28s} {v[0]:10.2f} {v[1]:10.2f}")
