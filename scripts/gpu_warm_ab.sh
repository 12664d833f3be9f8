#!/bin/bash
# GPU box: the driver's 20-step figure after W=5 / 50 / 200 warm-up steps, alternating, with the
# per-step host trace and rocm-smi clock samples (diagnostic: is a short run's interval set by the
# GPU's state before it?).
#   bash scripts/gpu_warm_ab.sh TAG
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=$1
O=gpurun_out; mkdir -p $O
( for k in $(seq 1 600); do echo "T $(date +%s.%N)"; timeout 5 rocm-smi --showclocks 2>/dev/null | grep -E 'sclk|mclk|fclk'; sleep 0.1; done ) > $O/clk_$TAG.txt 2>&1 &
CLK=$!
for i in 1 2; do
  for w in 5 50 200; do
    echo "B $(date +%s.%N) w=$w" >> $O/clk_$TAG.txt
    timeout -k 10 300 python -u bench.py --gpus 1 --steps 20 --warmup $w --no-dcn --no-cpu-baseline --no-c2 \
        > $O/warm_${TAG}_${w}_$i.json 2> $O/warm_${TAG}_${w}_$i.err || { echo "bench failed"; tail -20 $O/warm_${TAG}_${w}_$i.err; kill $CLK; exit 1; }
    echo "E $(date +%s.%N) w=$w" >> $O/clk_$TAG.txt
    echo "w=$w $(python scripts/bench_summary.py $O/warm_${TAG}_${w}_$i.json | cut -c1-400)"
  done
done
kill $CLK
echo EXIT 0
