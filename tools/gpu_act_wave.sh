# Wave-owned acting kernel on the GPU box: bit-identity tests, isolated launch timings of both
# launch-A kernels (MBK_ACT_WAVE=1 default / 0 = phase-split), then the headline bench.
#   bash tools/gpu_act_wave.sh <tag>
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; mkdir -p gpurun_out
tag=${1:-aw}
timeout -k 10 300 python -u -m pytest tests/test_gpu_act.py tests/test_gpu_fc.py tests/test_gpu_engine.py -x -q --timeout 120 --timeout-method thread \
  > gpurun_out/${tag}_act_tests.log 2>&1 || { tail -30 gpurun_out/${tag}_act_tests.log; exit 1; }
tail -2 gpurun_out/${tag}_act_tests.log
for w in 1 0; do
  MBK_ACT_WAVE=$w timeout -k 10 200 python tools/act_phases.py --envs 8192 --steps 30 \
    > gpurun_out/${tag}_phases_w$w.log 2>&1 || { tail -20 gpurun_out/${tag}_phases_w$w.log; exit 2; }
  echo "MBK_ACT_WAVE=$w"; grep -v amdgpu.ids gpurun_out/${tag}_phases_w$w.log
done
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/${tag}_bench.log 2>&1 || exit 3
tail -1 gpurun_out/${tag}_bench.log | cut -c1-300
