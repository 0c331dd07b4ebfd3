# Does the training trajectory differ between the fused stage backward kernels and the
# per-layer path? Settled bench twice each, alternating.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; mkdir -p gpurun_out
i=0
for v in "fused_pool_wgrad0=1 fused_pool_conv_bwd=1" "fused_pool_wgrad0=0 fused_pool_conv_bwd=0" \
         "fused_pool_wgrad0=1 fused_pool_conv_bwd=1" "fused_pool_wgrad0=0 fused_pool_conv_bwd=0"; do
  i=$((i+1))
  timeout -k 10 300 python tools/bench_variant.py $v -- --steps 20 --warmup 5 > gpurun_out/r5y_$i.log 2>&1 || { tail -20 gpurun_out/r5y_$i.log; exit 1; }
  python - <<PY
import json
d = json.loads([x for x in open("gpurun_out/r5y_$i.log") if x.startswith("{")][-1])
print("[$v]", d["value"], d["ms_per_step"], d["active_cells_per_env"], d["learner_phase_ms_rank0"]["bwd"], d["last_losses"]["entropy"])
PY
done
