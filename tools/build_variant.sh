#!/bin/bash
# Build liblightglue_mi355x.so from the sources of git revision $1 into $2 (same-box A/B runs:
# tools/ab_bench.sh).  Usage: bash tools/build_variant.sh HEAD ab/head.so
set -eu
rev=$1; out=$(realpath -m "$2")
root=$(cd "$(dirname "$0")/.." && pwd)
tmp=$(mktemp -d)
git -C "$root" archive "$rev" cs566-project-lightglue_amd/csrc include | tar -x -C "$tmp"
make -s -C "$tmp/cs566-project-lightglue_amd/csrc" -j8 OUT="$out" "$out"
rm -rf "$tmp"
echo "built $out from $rev"
