# One kernel iteration on the GPU box: the given GPU tests, then the isolated learner's timing and
# kernel table (tools/lt_ab.sh) and, optionally, counter passes of the named kernels.
#   [AB_A="--set enc.x=0" AB_B="--set enc.x=1"] bash tools/gpu_kernel_check.sh <tag> "<pytest -k expr>" [pmc kernel substrings]
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; mkdir -p gpurun_out
tag=$1; kexpr=$2; pmc=$3
if [ -n "$kexpr" ]; then
  timeout -k 10 300 python -u -m pytest tests/test_gpu_conv.py tests/test_gpu_learner_parity.py \
    tests/test_gpu_act.py tests/test_gpu_head.py -x -q --timeout 200 --timeout-method thread \
    -k "$kexpr" > gpurun_out/${tag}_tests.log 2>&1 || { tail -40 gpurun_out/${tag}_tests.log; exit 1; }
  tail -2 gpurun_out/${tag}_tests.log
fi
for act in 0.007 0.025; do
  timeout -k 10 200 python tools/learner_only.py --steps 5 --active $act > gpurun_out/${tag}_learner_$act.log 2>&1 || exit 2
  echo "learner (active $act): $(tail -1 gpurun_out/${tag}_learner_$act.log)"
done
if [ -n "$AB_A" ]; then
  LT_ARGS="--active 0.025" bash tools/lt_ab.sh ${tag} "$AB_A" "$AB_B" "$AB_A" "$AB_B" || exit 3
else
  LT_ARGS="--active 0.025" bash tools/lt_ab.sh ${tag} "MBK_NOP=0" || exit 3
fi
if [ -n "$pmc" ]; then
  bash tools/pmc_wait.sh ${tag} "$pmc" tools/learner_only.py --steps 2 || exit 4
  bash tools/pmc.sh ${tag} tools/learner_only.py --steps 2 || exit 5
  grep -E "$(echo $pmc | tr ',' '|')" gpurun_out/${tag}_pmc.md
  cat gpurun_out/${tag}_wait.md
fi
