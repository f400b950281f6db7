#!/bin/bash
# Build liblightglue_mi355x.so from the WORKING TREE with extra compile flags for single translation
# units into $1 (same-box A/B runs).  Each further argument is <stem>=<flags>:
#   bash tools/build_tu_flags.sh ab/x.so "gemm_h3=-mllvm -amdgpu-sched-strategy=max-ilp" "gemm=..."
set -eu
out=$(realpath -m "$1"); shift
root=$(cd "$(dirname "$0")/.." && pwd)
tmp=$(mktemp -d)
mkdir -p "$tmp/cs566-project-lightglue_amd"
cp -r "$root/cs566-project-lightglue_amd/csrc" "$tmp/cs566-project-lightglue_amd/"
rm -rf "$tmp/cs566-project-lightglue_amd/csrc/build"
cp -r "$root/include" "$tmp/"
vars=()
for a in "$@"; do vars+=("EXTRA_${a%%=*}=${a#*=}"); done
make -s -C "$tmp/cs566-project-lightglue_amd/csrc" -j8 OUT="$out" "${vars[@]}" "$out"
rm -rf "$tmp"
echo "built $out with $*"
