"""One line from a bench.py JSON record: xRT, step ms, batch-step s, and per-class live figures."""
import json
import sys

d = json.load(open(sys.argv[1]))
cl = d.get("roofline_classes") or {}
print("xRT %.1f  ms/step %.1f  batch_step_s %.3f  spec_s %.3f  fixup_s %.3f  launches %s  rows/launch %.1f  |  %s" % (
    d["value"], d["ms_per_step"], d["stages_s"].get("batch_step_s", 0), d["stages_s"].get("spec_s", 0),
    d["stages_s"].get("fixup_s", 0), d["counts"].get("batch_launches"),
    d["counts"].get("batch_rows", 0) / max(1, d["counts"].get("batch_launches", 1)),
    "  ".join("%s %.1fus x%d %s%.3f" % (k, v["avg_launch_us"], v["launches_est"], "", v["frac"]) for k, v in cl.items())))
