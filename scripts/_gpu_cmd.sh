cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out
bash scripts/gpu_check.sh || exit $?
T="timeout -k 10 120 python -u"
for r in 1 2; do
for b in ab/base dxrpathtracer_amd/lib; do
  DXRPT_KERNEL_LIB_DIR=$b $T scripts/time_frames.py --label "$b" --rounds 3 --frames 32 2>&1 | grep -v amdgpu.ids || exit 1
  DXRPT_KERNEL_LIB_DIR=$b $T scripts/time_frames.py --label "$b" --share 8 --rank 2 --rounds 3 --frames 32 2>&1 | grep -v amdgpu.ids || exit 1
  DXRPT_KERNEL_LIB_DIR=$b $T scripts/time_frames.py --label "$b" --config c4 --rounds 3 --frames 16 2>&1 | grep -v amdgpu.ids || exit 1
done; done
