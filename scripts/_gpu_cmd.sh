cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out
T="timeout -k 10 120 python -u"
for b in ab/nosun0 dxrpathtracer_amd/lib ab/ch1 ab/ch2 ab/ah1 ab/ah2 ab/nosun0 dxrpathtracer_amd/lib; do
  DXRPT_KERNEL_LIB_DIR=$b $T scripts/time_frames.py --rounds 3 --frames 32 --label "$b" 2>&1 | grep -v amdgpu.ids || exit 1
done
for b in ab/nosun0 dxrpathtracer_amd/lib; do
  DXRPT_KERNEL_LIB_DIR=$b $T scripts/time_frames.py --rounds 3 --frames 32 --max-path 2 --label "$b" 2>&1 | grep -v amdgpu.ids || exit 1
  DXRPT_KERNEL_LIB_DIR=$b $T scripts/time_frames.py --rounds 3 --frames 32 --share 8 --rank 2 --label "$b" 2>&1 | grep -v amdgpu.ids || exit 1
done
