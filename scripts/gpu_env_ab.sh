#!/bin/bash
# GPU box: environment-knob A/B (diagnostic): for each setting ("-" = none), kernel_ab.py (kernels
# alone) and step_modes2.py (steady-state intervals), alternating over the rounds.
#   bash scripts/gpu_env_ab.sh TAG ROUNDS "VAR=V VAR2=V2" ...
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=$1; R=$2; shift 2
O=gpurun_out; mkdir -p $O
for r in $(seq 1 $R); do
  for e in "$@"; do
    ev="$e"; [ "$ev" = "-" ] && ev=""
    env $ev timeout -k 10 150 python scripts/kernel_ab.py > $O/eab_k.json 2>> $O/eab_$TAG.err || { echo "kab [$e] failed"; tail -5 $O/eab_$TAG.err; exit 1; }
    env $ev timeout -k 10 300 python -u scripts/step_modes2.py --steps 300 > $O/eab_m.json 2>> $O/eab_$TAG.err || { echo "modes [$e] failed"; tail -5 $O/eab_$TAG.err; exit 1; }
    echo "[$e] r$r kernels $(cut -c1-220 $O/eab_k.json)"
    echo "[$e] r$r modes $(python -c 'import json,sys; d=json.load(open(sys.argv[1])); print({k:v for k,v in d["rep1"].items() if "host" not in k})' $O/eab_m.json)"
  done
done
echo EXIT 0
