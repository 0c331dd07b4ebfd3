set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_conv.py -q --timeout 200 --timeout-method thread > gpurun_out/t7.log 2>&1
rc=$?; tail -2 gpurun_out/t7.log; grep -E "^E |FAILED" gpurun_out/t7.log | head -20; if [ $rc -gt 1 ]; then exit $rc; fi
for v in "MBK_FUSED_RES=0" "MBK_FUSED_RES=1"; do
  env $v timeout -k 10 200 python tools/microbench.py --E "" --learn_B 8192 --iters 20 > gpurun_out/ab.log 2>&1 || exit $?
  echo "$v $(grep learner_update gpurun_out/ab.log | cut -c1-130)"
done
