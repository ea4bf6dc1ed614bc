#!/bin/bash
# r03: split-schedule budgets and part counts once frames overlap.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
T="timeout -k 10 200 python -u scripts/time_frames.py --rounds 3 --frames 32"
run() { $T "$@" 2>&1 | grep -v amdgpu.ids || exit 1; }
run --config metric --label default
for ho in 5 6 7; do for to in 6 7 8; do
  run --config metric --msplit 1 --parts 1 --occ $ho --tail-occ $to --label split1
done; done
run --config c4 --msplit 1 --parts 1 --occ 5 --label split1
run --config c2 --msplit 1 --parts 1 --occ 5 --label split1
run --config c2 --msplit 1 --parts 1 --occ 7 --label split1
run --config metric --share 2 --rank 1 --msplit 1 --parts 1 --label split1
run --config c5 --share 8 --rank 3 --msplit 1 --parts 1 --label split1
run --config c3 --msplit 1 --parts 1 --label split1
run --config c3 --msplit 1 --parts 2 --label split2
run --config c3 --share 8 --rank 3 --label default
run --config c3 --share 8 --rank 3 --msplit 1 --parts 1 --label split1
run --config c3 --share 8 --rank 3 --msplit 1 --parts 2 --label split2
