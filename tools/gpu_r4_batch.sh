# One GPU call: acting-kernel tests + phases + bench (tools/gpu_act_wave.sh), the learner parity
# and DP-equality tests, and the active-cell sweep. Stops at the first crash / time limit.
#   bash tools/gpu_r4_batch.sh <tag>
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; mkdir -p gpurun_out
tag=${1:-b}
bash tools/gpu_act_wave.sh $tag || exit $?
timeout -k 10 400 python -u -m pytest tests/test_gpu_learner_parity.py tests/test_gpu_dp_equality.py \
  -x -q -s --timeout 300 --timeout-method thread > gpurun_out/${tag}_lp.log 2>&1
rc=$?
grep -E "passed|failed|bf16 floor|Error|assert" gpurun_out/${tag}_lp.log | tail -40
if [ $rc -gt 1 ]; then exit $rc; fi
timeout -k 10 300 python tools/active_sweep.py --envs 8192 --cpu_envs 128 --cpu_steps 600 \
  > gpurun_out/${tag}_sweep.log 2>&1 || exit $?
grep what gpurun_out/${tag}_sweep.log
