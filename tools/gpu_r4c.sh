# One GPU call: head tests, learner trace, acting phases with rows in pinned host memory vs
# HBM (fused / B forms), and the bench per head form twice (run-to-run spread).
#   bash tools/gpu_r4c.sh <tag>
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; mkdir -p gpurun_out
tag=${1:-r4c}
timeout -k 10 300 python -u -m pytest tests/test_gpu_head.py -x -q --timeout 200 --timeout-method thread \
  > gpurun_out/${tag}_head_tests.log 2>&1 || { tail -30 gpurun_out/${tag}_head_tests.log; exit 1; }
tail -1 gpurun_out/${tag}_head_tests.log
bash tools/lt_ab.sh ${tag} "MBK_NOP=0" || exit 2
grep -E "head_|pool_bwd" gpurun_out/${tag}_lt1.md
for f in 1 0; do for dr in "" "--device_rows"; do
  MBK_ACT_FUSED=$f timeout -k 10 200 python tools/act_phases.py --envs 8192 --steps 30 $dr \
    > gpurun_out/${tag}_ph_f${f}${dr}.log 2>&1 || { tail -20 gpurun_out/${tag}_ph_f${f}${dr}.log; exit 3; }
  echo "== fused=$f $dr"; grep -E "launch A|first tile|rows|decode|barrier|FC|head" gpurun_out/${tag}_ph_f${f}${dr}.log
done; done
for rep in 1 2; do for form in auto 1 0; do
  if [ $form = auto ]; then env_set=""; else env_set="MBK_ACT_FUSED=$form"; fi
  env $env_set timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/${tag}_bench_${form}_$rep.log 2>&1 || exit 4
  python - "$form" gpurun_out/${tag}_bench_${form}_$rep.log <<'PY'
import json, sys
r = json.loads(open(sys.argv[2]).read().strip().splitlines()[-1])
a = r.get("actor_stats_per_rank", [{}])[0]
print(sys.argv[1], r["value"], r["ms_per_step"], r.get("learner_phase_ms_rank0"), {k: a.get(k) for k in
      ("act_head_in_A_frac", "active_cells_per_env", "gpu_phase_ms", "env_phase_ms")})
PY
done; done
