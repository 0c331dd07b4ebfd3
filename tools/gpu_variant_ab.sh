# Does the training trajectory (and the settled bench) differ between two HipEncoder variant
# sets? The settled bench twice each, alternating (tools/bench_variant.py; profile 40 ran the
# fused stage backward kernels against the per-layer path as tag r5y).
#   bash tools/gpu_variant_ab.sh <tag> "<attr=v ...>" "<attr=v ...>"
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; mkdir -p gpurun_out
tag=$1; A=$2; B=$3
i=0
for v in "$A" "$B" "$A" "$B"; do
  i=$((i+1))
  timeout -k 10 300 python tools/bench_variant.py $v -- --steps 20 --warmup 5 > gpurun_out/${tag}_$i.log 2>&1 || { tail -20 gpurun_out/${tag}_$i.log; exit 1; }
  python - "$v" gpurun_out/${tag}_$i.log <<'PY'
import json, sys
d = json.loads([x for x in open(sys.argv[2]) if x.startswith("{")][-1])
print(f"[{sys.argv[1]}]", d["value"], d["ms_per_step"], d["active_cells_per_env"],
      d["learner_phase_ms_rank0"]["bwd"], d["last_losses"]["entropy"])
PY
done
