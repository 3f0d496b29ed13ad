#!/bin/bash
# Build the mmseq library of a git revision into ab/libmmseq_<name>.so (A/B timing against the
# working tree in one GPU process: MMSEQ_BENCH_LIB=ab/libmmseq_<name>.so). usage: ab_build.sh REV NAME
set -e
REV=$1; NAME=$2
ROOT=$(cd "$(dirname "$0")/.." && pwd)
W=$(mktemp -d /tmp/abbuild.XXXX)
mkdir -p "$W/include" "$W/pkg"
git -C "$ROOT" archive "$REV" include multimodal_sequencing_amd/csrc | tar -x -C "$W/pkg"
cp -r "$W/pkg/include/." "$W/include/"
mv "$W/pkg/multimodal_sequencing_amd/csrc" "$W/pkg/csrc"
make -C "$W/pkg/csrc" -j8 OUT="$W/lib.so" > "$W/build.log" 2>&1 || { tail -20 "$W/build.log"; exit 1; }
mkdir -p "$ROOT/ab"
cp "$W/lib.so" "$ROOT/ab/libmmseq_$NAME.so"
rm -rf "$W"
echo "ab/libmmseq_$NAME.so"
