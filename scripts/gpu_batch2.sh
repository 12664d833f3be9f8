#!/bin/bash
# GPU box: suite + smoke + bench + rocprofv3 (gpu_r3.sh), per-kernel A/B vs the `head` variant,
# the step timeline.   bash scripts/gpu_batch2.sh TAG
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=${1:-run}
bash scripts/gpu_r3.sh $TAG && bash scripts/gpu_kernel_ab.sh $TAG head && bash scripts/gpu_timeline.sh $TAG
rc=$?
echo "EXIT $rc"
exit $rc
