#!/bin/bash
# Interleaved A/B of library env knobs on tools/bench_configs.py configs (diagnostic tooling).
#   tools/ab_env.sh CONFIGS REPEATS "ENV1=a ENV2=b" "ENV1=c" ...
cfgs=$1; reps=$2; shift 2
for i in $(seq "$reps"); do
  for cfg in "$@"; do
    env $cfg python3 tools/bench_configs.py --configs "$cfgs" --steps 20 --warmup 3 2>/dev/null |
      python3 -c "import sys, json
for l in sys.stdin:
    if l.startswith('{'):
        d = json.loads(l); print(json.dumps({'env': '$cfg', 'config': d['config'], 'ms': d['ms']}))"
  done
done
