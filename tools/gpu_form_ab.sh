# Per-step head form on the GPU box: acting tests (every form incl. the engine's mixed
# choice), then the headline bench with the engine's choice (auto) and each form forced.
#   bash tools/gpu_form_ab.sh <tag>
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; mkdir -p gpurun_out
tag=${1:-fa}
timeout -k 10 300 python -u -m pytest tests/test_gpu_act.py -x -q --timeout 120 --timeout-method thread \
  > gpurun_out/${tag}_act_tests.log 2>&1 || { tail -30 gpurun_out/${tag}_act_tests.log; exit 1; }
tail -1 gpurun_out/${tag}_act_tests.log
for form in auto 1 0; do
  if [ $form = auto ]; then env_set=""; else env_set="MBK_ACT_FUSED=$form"; fi
  env $env_set timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/${tag}_bench_$form.log 2>&1 || exit 3
  python - "$form" gpurun_out/${tag}_bench_$form.log <<'PY'
import json, sys
r = json.loads(open(sys.argv[2]).read().strip().splitlines()[-1])
a = r.get("actor_stats_per_rank", [{}])[0]
print(sys.argv[1], r["value"], r["ms_per_step"], {k: a.get(k) for k in
      ("act_head_in_A_frac", "active_cells_per_env", "gpu_phase_ms", "env_phase_ms", "env_worker_busy_frac")})
PY
done
