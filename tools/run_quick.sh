set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
bash tools/gpu_suite.sh s1 || exit $?
timeout -k 10 300 python tools/aten_audit.py --arch impala_flat --size 16 --batch 2048 > gpurun_out/audit_i.log 2>&1 || exit $?
tail -12 gpurun_out/audit_i.log
