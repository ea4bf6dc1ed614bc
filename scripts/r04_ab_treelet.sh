#!/bin/bash
# r04 A/B: treelet-restructured BVH (Karras & Aila 2013; subtrees holding alpha-tested triangles left as built)
# before the BVH8 collapse: 0 / 1 (shipped) / 2 passes through DXRPT_OPT_TREELET_PASSES on the in-tree build
# (the recorded run, profiles/r04_ab_treelet.txt, used builds with -DDXRPT_TREELET_PASSES=n instead).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -c "import torch; torch.zeros(1, device='cuda')" || exit 1
T="timeout -k 10 150 python -u scripts/time_frames.py --rounds 3"
for cfg in "--config metric" "--config c2" "--config c3 --frames 16" "--config c4" "--config c5 --frames 8" "--config metric --share 8 --rank 2" "--config metric --share 8 --rank 7"; do
  for r in 1 2; do
    for n in 0 1 2; do
      $T $cfg --opt TREELET_PASSES=$n --label tl$n 2>> gpurun_out/ab_treelet.err
      rc=$?; [ $rc -ne 0 ] && { echo "tl$n $cfg rc=$rc"; [ $rc -gt 1 ] && exit $rc; }
    done
  done
done
exit 0
