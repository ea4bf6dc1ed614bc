#!/bin/bash
# Host-code sanitizer run (CPU only): the host library's sources (scenes, FBX, DDS, PNG, JPEG, Hosek sky,
# lightmap charts) built with AddressSanitizer + UndefinedBehaviorSanitizer together with
# csrc/tools/host_fuzz.cpp, which loads the reference's own texture and model files and seeded corrupted
# copies of them (truncations, byte flips).  Needs /root/reference (this container); outputs under
# /tmp/dxrpt_asan.  Usage: scripts/asan_host.sh [mutants per file, default 64]
set -e
cd "$(dirname "$0")/../dxrpathtracer_amd/csrc"
OUT=/tmp/dxrpt_asan
mkdir -p $OUT
SAN="-fsanitize=address,undefined -fno-sanitize-recover=undefined -fno-omit-frame-pointer -g -O1"
g++ -std=c++17 $SAN -ffp-contract=off -o $OUT/host_fuzz tools/host_fuzz.cpp host/*.cpp -lz -lpthread
# the scene tests' own built-in scenes (proxies, BoxTest) through the same sanitized library
FILES=$(find /root/reference/Content -type f \( -iname "*.png" -o -iname "*.jpg" -o -iname "*.jpeg" -o -iname "*.dds" -o -iname "*.fbx" \) | sort)
ASAN_OPTIONS=detect_leaks=1:abort_on_error=1 UBSAN_OPTIONS=print_stacktrace=1 \
  $OUT/host_fuzz --mutants ${1:-64} --tmp $OUT $FILES
echo "asan_host: clean"
