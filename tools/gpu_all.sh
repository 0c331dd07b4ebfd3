# Full GPU check in one call: every GPU test, the headline bench, then the GridNet (config 2)
# measurements and a kernel profile of one GridNet learner update. Stops at the first crash.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; mkdir -p gpurun_out
tag=${1:-all}
timeout -k 10 600 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > gpurun_out/${tag}_pytest.log 2>&1
rc=$?
tail -3 gpurun_out/${tag}_pytest.log
if [ $rc -gt 1 ]; then echo "pytest rc=$rc: stopping"; exit $rc; fi
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/${tag}_bench.log 2>&1 || exit $?
tail -1 gpurun_out/${tag}_bench.log | cut -c1-300
timeout -k 10 200 python tools/learner_only.py --arch gridnet --size 10 --steps 3 > gpurun_out/${tag}_gn_lt.log 2>&1 || exit $?
cat gpurun_out/${tag}_gn_lt.log
timeout -k 10 200 python tools/microbench.py --arch gridnet --size 10 --E 8192 --iters 20 --no_learner > gpurun_out/${tag}_gn_micro.log 2>&1 || exit $?
grep '"what"' gpurun_out/${tag}_gn_micro.log
timeout -k 10 300 python bench.py --steps 10 --warmup 3 --size 10 --arch gridnet > gpurun_out/${tag}_gn_bench.log 2>&1 || exit $?
tail -1 gpurun_out/${tag}_gn_bench.log | cut -c1-300
MBK_PROF_SEQ=120 bash tools/prof.sh ${tag}_gn_prof tools/learner_only.py --arch gridnet --size 10 --steps 1 || exit $?
exit $rc
