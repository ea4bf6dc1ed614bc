cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out
bash scripts/gpu_check.sh || exit $?
T="timeout -k 10 120 python -u"
for r in 1 2; do for b in ab/head dxrpathtracer_amd/lib; do
  DXRPT_KERNEL_LIB_DIR=$b $T scripts/time_frames.py --rounds 3 --frames 32 --label $b 2>&1 | grep -v amdgpu.ids || exit 1
done; done
for b in ab/head dxrpathtracer_amd/lib; do
  DXRPT_KERNEL_LIB_DIR=$b $T scripts/time_frames.py --rounds 3 --frames 32 --config c2 --label $b 2>&1 | grep -v amdgpu.ids || exit 1
  DXRPT_KERNEL_LIB_DIR=$b $T scripts/time_frames.py --rounds 3 --frames 32 --config c4 --label $b 2>&1 | grep -v amdgpu.ids || exit 1
  for s in "8 1" "8 2" "8 6" "4 1" "2 1"; do set -- $s
    DXRPT_KERNEL_LIB_DIR=$b $T scripts/time_frames.py --rounds 3 --frames 32 --share $1 --rank $2 --label $b 2>&1 | grep -v amdgpu.ids || exit 1
  done
done
