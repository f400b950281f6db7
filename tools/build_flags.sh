#!/bin/bash
# Build liblightglue_mi355x.so from the WORKING TREE with extra compile flags into $1 (same-box A/B
# runs).  Usage: bash tools/build_flags.sh ab/x.so -DLG_TG_BK=32 ...
set -eu
out=$(realpath -m "$1"); shift
root=$(cd "$(dirname "$0")/.." && pwd)
tmp=$(mktemp -d)
mkdir -p "$tmp/cs566-project-lightglue_amd"
cp -r "$root/cs566-project-lightglue_amd/csrc" "$tmp/cs566-project-lightglue_amd/"
rm -rf "$tmp/cs566-project-lightglue_amd/csrc/build"
cp -r "$root/include" "$tmp/"
make -s -C "$tmp/cs566-project-lightglue_amd/csrc" -j8 OUT="$out" EXTRA="$*" "$out"
rm -rf "$tmp"
echo "built $out with $*"
