# Bitmap rows: acting tests (bitmap vs masks every step, learner update with / without it),
# learner trace, bench.
#   bash tools/gpu_r4g.sh <tag>
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; mkdir -p gpurun_out
tag=${1:-r4g}
timeout -k 10 400 python -u -m pytest tests/test_gpu_act.py tests/test_gpu_head.py tests/test_gpu_engine.py -x -q --timeout 200 --timeout-method thread \
  > gpurun_out/${tag}_tests.log 2>&1 || { tail -30 gpurun_out/${tag}_tests.log; exit 1; }
tail -1 gpurun_out/${tag}_tests.log
for rep in 1 2; do
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/${tag}_bench$rep.log 2>&1 || exit 3
python - gpurun_out/${tag}_bench$rep.log <<'PY'
import json, sys
r = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
a = r.get("actor_stats_per_rank", [{}])[0]
print("bench", r["value"], r["ms_per_step"], r.get("learner_phase_ms_rank0"), a.get("gpu_phase_ms"))
PY
done
