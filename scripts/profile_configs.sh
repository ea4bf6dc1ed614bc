#!/bin/bash
# scripts/profile.sh for several configs, each summarised into profiles/<round>_* (pmc_summary.py).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
RND=${RND:-r04}
for c in ${CONFIGS:-metric c3 c5}; do
  case $c in
    metric) cfg="sponza-proxy 1920x1080 L=3";; c2) cfg="sponza-proxy 1280x720 L=3";; c3) cfg="sponza-proxy 1920x1080 L=8";;
    c4) cfg="suntemple-proxy 1920x1080 L=3";; c5) cfg="sponza-proxy 3840x2160 L=6";;
  esac
  CONFIG=$c STEPS=${STEPS:-24} bash scripts/profile.sh > gpurun_out/profile_$c.log 2>&1 || { echo "profile $c failed"; tail -5 gpurun_out/profile_$c.log; exit 1; }
  PMC_CONFIG_TAG=$c PMC_CONFIG="$cfg" python3 scripts/pmc_summary.py gpurun_out/prof_$c $RND || exit 1
done
# only gpurun_out/ comes back from the GPU box: the summaries travel with it
mkdir -p gpurun_out/profiles && cp profiles/${RND}_launch_* profiles/${RND}_kernel_* gpurun_out/profiles/
