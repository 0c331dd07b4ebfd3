set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)}; mkdir -p gpurun_out
for rep in 1 2; do
for v in default spec40 spec48; do
  lib=""; [ "$v" = default ] || lib="--lib variants/$v"
  timeout -k 10 240 python tools/act_phases.py --envs 8192 --steps 40 --spread --settled_rows $lib > gpurun_out/r6spec_$v.log 2>&1 || { tail -20 gpurun_out/r6spec_$v.log; exit 4; }
  echo "$v: $(grep 'launch A' gpurun_out/r6spec_$v.log) | $(grep 'barrier' gpurun_out/r6spec_$v.log)"
done
done
grep "settled rows" gpurun_out/r6spec_default.log
