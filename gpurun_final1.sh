cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp
TAG=r06final STEPS=20 bash scripts/gpu_check.sh || exit $?
bash scripts/bench_configs.sh || exit 1
bash scripts/shares_all_ranks.sh > gpurun_out/shares_all_ranks_final.txt 2>&1; echo "shares rc=$?"
