"""Print one line per bench JSON in a sweep file (tools/pipeline_sweep.sh)."""
import json
import sys

for line in open(sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/sweep/pipeline.jsonl"):
    if line.startswith("=="):
        print(line.strip())
        continue
    d = json.loads(line)
    print(round(d["value"] / 1e6, 3), round(d["ms_per_step"], 3),
          round(d["roofline"]["frac"], 4), d["stages_ms"])
