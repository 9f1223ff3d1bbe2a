#!/bin/bash
# Build experiment variants of libptamd.so into variants/<name>/ (git-ignored; they travel to the
# GPU box with the snapshot). Usage: tools/build_variants.sh name "DEVFLAGS" [name "DEVFLAGS" ...]
# Select one at run time with PT_LIB=variants/<name>/libptamd.so.
set -e
ROOT=$(cd "$(dirname "$0")/.." && pwd)
while [ $# -ge 2 ]; do
  d=$ROOT/variants/$1
  mkdir -p $d/build
  make -s -C $ROOT/cudapathtracer_amd/csrc -j8 OUT=$d/libptamd.so OBJDIR=$d/build/ DEVFLAGS="$2"
  echo "built $d/libptamd.so ($2)"
  shift 2
done
