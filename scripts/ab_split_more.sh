cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
T="timeout -k 10 180 python -u scripts/time_frames.py --rounds 3 --frames 24"
for L in 4 5; do
  $T --config metric --max-path $L --msplit 0 --label single || exit 1
  $T --config metric --max-path $L --msplit 1 --occ 6 --tail-occ 7 --label split || exit 1
  $T --config metric --max-path $L --msplit 1 --occ 5 --tail-occ 7 --label split || exit 1
done
$T --config c5 --share 8 --rank 3 --label single-ordered || exit 1
$T --config c5 --share 8 --rank 3 --wave-order 0 --label single-pathorder || exit 1
$T --config c5 --share 8 --rank 3 --wave-order 0 --msplit 1 --occ 6 --tail-occ 7 --label split || exit 1
$T --config c3 --share 8 --rank 3 --label single-ordered || exit 1
$T --config c3 --share 8 --rank 3 --wave-order 0 --lanes 64 --msplit 1 --occ 6 --tail-occ 7 --label split || exit 1
for c in metric c3 c4; do
  DXRPT_KERNEL_LIB_DIR=ab/stage $T --config $c --label stage || exit 1
  for o in 6 5; do DXRPT_KERNEL_LIB_DIR=ab/stage $T --config $c --occ $o --label stage || exit 1; done
done
