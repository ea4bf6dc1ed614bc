#!/bin/bash
# Every BASELINE.json config through bench.py on one GPU (the metric config with its CPU baseline, the
# others without), one JSON line each -> gpurun_out/configs.jsonl.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
: > gpurun_out/configs.jsonl
for c in metric c2 c3 c4 c5; do
  extra="--no-cpu-baseline"; [ $c = metric ] && extra=""
  timeout -k 10 400 python bench.py --config $c --steps 32 --warmup 5 $extra >> gpurun_out/configs.jsonl 2> gpurun_out/bench_$c.err \
    || { echo "bench $c failed"; tail -5 gpurun_out/bench_$c.err; exit 1; }
  echo "$c ok"
done
