# Dynamic tile queue: acting tests, bench x2, timeline.
#   bash tools/gpu_r4k.sh <tag>
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; mkdir -p gpurun_out
tag=${1:-r4k}
timeout -k 10 300 python -u -m pytest tests/test_gpu_act.py -x -q --timeout 120 --timeout-method thread \
  > gpurun_out/${tag}_tests.log 2>&1 || { tail -30 gpurun_out/${tag}_tests.log; exit 1; }
tail -1 gpurun_out/${tag}_tests.log
timeout -k 10 200 python tools/act_phases.py --envs 8192 --steps 30 > gpurun_out/${tag}_ph.log 2>&1 || { tail -20 gpurun_out/${tag}_ph.log; exit 2; }
grep -E "launch A|first tile" gpurun_out/${tag}_ph.log
for rep in 1 2; do
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/${tag}_bench$rep.log 2>&1 || exit 3
python - gpurun_out/${tag}_bench$rep.log <<'PY'
import json, sys
r = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
a = r.get("actor_stats_per_rank", [{}])[0]
print("bench", r["value"], r["ms_per_step"], r.get("learner_phase_ms_rank0"), a.get("gpu_phase_ms"))
PY
done
export TMPDIR=/tmp
rm -rf /tmp/${tag}_tl
(cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace -d /tmp/${tag}_tl -o run --output-format csv \
  -- python $R/bench.py --steps 12 --warmup 4) > gpurun_out/${tag}_tl_bench.log 2>&1 || exit 4
python tools/timeline.py /tmp/${tag}_tl > gpurun_out/${tag}_timeline.txt 2>&1 || exit 5
head -10 gpurun_out/${tag}_timeline.txt
