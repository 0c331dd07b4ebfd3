# 12-wide stage fusion: conv tests, config 4 bench + learner trace.
#   bash tools/gpu_r4i.sh <tag>
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; mkdir -p gpurun_out
tag=${1:-r4i}
timeout -k 10 300 python -u -m pytest tests/test_gpu_conv.py tests/test_gpu_obs_mask.py -x -q -k "stage or conv0_row or res_ or wgrad or mask" --timeout 200 --timeout-method thread \
  > gpurun_out/${tag}_tests.log 2>&1 || { tail -30 gpurun_out/${tag}_tests.log; exit 1; }
tail -1 gpurun_out/${tag}_tests.log
timeout -k 10 300 python bench.py --steps 10 --warmup 3 --size 24 --arch impala_deep > gpurun_out/${tag}_c4.log 2>&1 || exit 2
python - gpurun_out/${tag}_c4.log <<'PY'
import json, sys
r = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print("c4", r["value"], r["ms_per_step"], r.get("learner_phase_ms_rank0"))
PY
timeout -k 10 300 python tools/learner_only.py --arch impala_deep --size 24 --steps 3 > gpurun_out/${tag}_c4_learner.log 2>&1 || exit 3
tail -1 gpurun_out/${tag}_c4_learner.log
