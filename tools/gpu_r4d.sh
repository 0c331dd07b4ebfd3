# One GPU call: acting tests (row staging included), phases with staged rows, and the bench
# with / without the row staging (MBK_ACT_ROWS_DEV) twice each.
#   bash tools/gpu_r4d.sh <tag>
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; mkdir -p gpurun_out
tag=${1:-r4d}
timeout -k 10 300 python -u -m pytest tests/test_gpu_act.py tests/test_gpu_engine.py -x -q --timeout 120 --timeout-method thread \
  > gpurun_out/${tag}_act_tests.log 2>&1 || { tail -30 gpurun_out/${tag}_act_tests.log; exit 1; }
tail -1 gpurun_out/${tag}_act_tests.log
for v in "--staged" ""; do
  timeout -k 10 200 python tools/act_phases.py --envs 8192 --steps 30 $v > gpurun_out/${tag}_ph$v.log 2>&1 \
    || { tail -20 gpurun_out/${tag}_ph$v.log; exit 3; }
  echo "== $v"; grep -E "launch A|first tile|rows|decode" gpurun_out/${tag}_ph$v.log
done
for rep in 1 2; do for rd in 1 0; do
  MBK_ACT_ROWS_DEV=$rd timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/${tag}_bench_rd${rd}_$rep.log 2>&1 || exit 4
  python - "rows_dev=$rd" gpurun_out/${tag}_bench_rd${rd}_$rep.log <<'PY'
import json, sys
r = json.loads(open(sys.argv[2]).read().strip().splitlines()[-1])
a = r.get("actor_stats_per_rank", [{}])[0]
print(sys.argv[1], r["value"], r["ms_per_step"], r.get("learner_phase_ms_rank0"), {k: a.get(k) for k in
      ("act_head_in_A_frac", "gpu_phase_ms", "env_phase_ms")})
PY
done; done
# config 5 (self-play league group) on the fused acting path, bf16
timeout -k 10 300 python bench.py --steps 15 --warmup 4 --selfplay_groups 1 > gpurun_out/${tag}_c5.log 2>&1 || exit 5
echo "c5 bf16: $(tail -1 gpurun_out/${tag}_c5.log | cut -c1-200)"
# config 4 (24x24 deep encoder) and config 2 through the engine: graph path, sparse row I/O
timeout -k 10 300 python bench.py --steps 10 --warmup 3 --size 24 --arch impala_deep > gpurun_out/${tag}_c4.log 2>&1 || exit 6
echo "c4: $(tail -1 gpurun_out/${tag}_c4.log | cut -c1-200)"
timeout -k 10 300 python bench.py --steps 10 --warmup 3 --size 10 --arch gridnet > gpurun_out/${tag}_c2e.log 2>&1 || exit 7
echo "c2 engine: $(tail -1 gpurun_out/${tag}_c2e.log | cut -c1-200)"
# learner: pool backward folded into the stage conv's staging, per stage set
bash tools/lt_ab.sh ${tag}pb "MBK_FUSED_POOL_BWD=0" "MBK_FUSED_POOL_BWD=s12" "MBK_FUSED_POOL_BWD=s1" || exit 8
