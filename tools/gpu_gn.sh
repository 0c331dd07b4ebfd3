set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_pixconv.py tests/test_gpu_gridnet.py -x -v --timeout 200 --timeout-method thread > gpurun_out/gn1_pytest.log 2>&1; rc=$?
tail -25 gpurun_out/gn1_pytest.log
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 200 python tools/learner_only.py --arch gridnet --size 10 --steps 3 > gpurun_out/gn1_lt.log 2>&1 || exit $?
cat gpurun_out/gn1_lt.log
bash tools/prof.sh gn1_prof tools/learner_only.py --arch gridnet --size 10 --steps 2 || exit $?
head -30 gpurun_out/gn1_prof_summary.md
