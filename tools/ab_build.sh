#!/bin/bash
# Build the mmseq library of a git revision (or of the working tree: REV = WORKTREE) into
# ab/libmmseq_<name>.so, optionally with extra compiler defines (A/B timing in one GPU call:
# MMSEQ_BENCH_LIB=ab/libmmseq_<name>.so). usage: ab_build.sh REV NAME [DEFS...]
# (FLAGS as in csrc/Makefile since round 3; builds of older revisions get -fno-slp-vectorize too)
set -e
REV=$1; NAME=$2; shift 2; DEFS="$*"
ROOT=$(cd "$(dirname "$0")/.." && pwd)
W=$(mktemp -d /tmp/abbuild.XXXX)
mkdir -p "$W/include" "$W/pkg"
if [ "$REV" = WORKTREE ]; then
  (cd "$ROOT" && tar -c include multimodal_sequencing_amd/csrc) | tar -x -C "$W/pkg"
else
  git -C "$ROOT" archive "$REV" include multimodal_sequencing_amd/csrc | tar -x -C "$W/pkg"
fi
cp -r "$W/pkg/include/." "$W/include/"
mv "$W/pkg/multimodal_sequencing_amd/csrc" "$W/pkg/csrc"
make -C "$W/pkg/csrc" -j8 OUT="$W/lib.so" FLAGS="-O3 -fPIC -std=c++17 --offload-arch=gfx950 -Wno-unused-result -fno-slp-vectorize $DEFS" > "$W/build.log" 2>&1 || { tail -20 "$W/build.log"; exit 1; }
mkdir -p "$ROOT/ab"
cp "$W/lib.so" "$ROOT/ab/libmmseq_$NAME.so"
rm -rf "$W"
echo "ab/libmmseq_$NAME.so"
