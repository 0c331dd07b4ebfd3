# Acting-step evidence on the GPU box: isolated launch timings + phase stamps of the fused
# policy step (tools/act_phases.py), then MFMA / LDS / HBM counter passes and the stall passes
# for act_trunk_kernel and head_act_kernel. Stops at the first failure.
#   bash tools/gpu_act_pmc.sh <tag>
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; mkdir -p gpurun_out
tag=${1:-act}
timeout -k 10 240 python tools/act_phases.py --envs 8192 --steps 30 > gpurun_out/${tag}_phases.log 2>&1 || exit $?
cat gpurun_out/${tag}_phases.log
bash tools/pmc.sh ${tag} tools/act_phases.py --envs 8192 --steps 10 || exit $?
bash tools/pmc_wait.sh ${tag} act_trunk,head_act tools/act_phases.py --envs 8192 --steps 10 || exit $?
cat gpurun_out/${tag}_pmc.md gpurun_out/${tag}_wait.md
