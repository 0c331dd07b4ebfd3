# GridNet (BASELINE config 2) check on the GPU box: pixconv / GridNet GPU tests, learner update
# time (sparse and dense logits layer), policy-step graph, the config-2 engine bench and a
# per-dispatch profile of one learner update.   bash tools/gpu_gn.sh <tag>
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; mkdir -p gpurun_out
tag=${1:-gs}
timeout -k 10 400 python -u -m pytest tests/test_gpu_pixconv.py tests/test_gpu_gridnet.py -x -v --timeout 200 --timeout-method thread > gpurun_out/${tag}_pytest.log 2>&1 || { tail -40 gpurun_out/${tag}_pytest.log; exit 1; }
tail -2 gpurun_out/${tag}_pytest.log
timeout -k 10 200 python tools/learner_only.py --arch gridnet --size 10 --steps 3 > gpurun_out/${tag}_lt.log 2>&1 || exit $?
cat gpurun_out/${tag}_lt.log
MBK_GRID_SPARSE=0 timeout -k 10 200 python tools/learner_only.py --arch gridnet --size 10 --steps 3 > gpurun_out/${tag}_lt_dense.log 2>&1 || exit $?
cat gpurun_out/${tag}_lt_dense.log
timeout -k 10 200 python tools/microbench.py --arch gridnet --size 10 --E 8192 --iters 20 --no_learner > gpurun_out/${tag}_micro.log 2>&1 || exit $?
grep '"what"' gpurun_out/${tag}_micro.log
timeout -k 10 300 python bench.py --steps 10 --warmup 3 --size 10 --arch gridnet > gpurun_out/${tag}_bench.log 2>&1 || exit $?
tail -1 gpurun_out/${tag}_bench.log | cut -c1-300
MBK_PROF_SEQ=120 bash tools/prof.sh ${tag}_prof tools/learner_only.py --arch gridnet --size 10 --steps 1 || exit $?
