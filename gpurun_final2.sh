cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp
CONFIGS="metric c2 c4 c3 c5" BENCH=0 RND=r06 bash scripts/final_profiles.sh || exit 1
bash scripts/debug_build_run.sh
