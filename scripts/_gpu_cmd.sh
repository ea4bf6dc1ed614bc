cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out
bash scripts/gpu_check.sh || exit $?
T="timeout -k 10 120 python -u"
for L in bands blocks; do for r in 0 1 2 3 4 5 6 7; do
  $T scripts/time_frames.py --share 8 --rank $r --layout $L --rounds 3 --frames 32 --label "s8 $L" 2>&1 | grep -v amdgpu.ids || exit 1
done; done
