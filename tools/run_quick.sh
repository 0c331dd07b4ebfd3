set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_train_entry.py tests/test_gpu_engine.py tests/test_gpu_agent_api.py -q --timeout 200 --timeout-method thread -k "not improves" > gpurun_out/t4.log 2>&1
rc=$?; tail -3 gpurun_out/t4.log; grep -E "^E |FAILED" gpurun_out/t4.log | head -20; if [ $rc -gt 1 ]; then exit $rc; fi
bash tools/prof.sh pol tools/microbench.py --E 8192 --learn_B "" --iters 40 --policy_eager || exit $?
sed -n 1,28p gpurun_out/pol_summary.md
