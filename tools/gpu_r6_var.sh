# Isolated acting launches for the default library and variants (tools/variant.py).
#   bash tools/gpu_r6_var.sh <tag> <variant>...
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)}; mkdir -p gpurun_out
tag=$1; shift
for v in default "$@"; do
  lib=""; [ "$v" = default ] || lib="--lib variants/$v"
  for sp in "" "--spread"; do
    timeout -k 10 240 python tools/act_phases.py --envs 8192 --steps 30 $sp $lib > gpurun_out/${tag}_${v}$sp.log 2>&1 || { tail -20 gpurun_out/${tag}_${v}$sp.log; exit 4; }
    echo "$v spread=$sp: $(grep 'launch A' gpurun_out/${tag}_${v}$sp.log)"
  done
done
