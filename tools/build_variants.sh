#!/bin/bash
# Build experiment variants of libptamd.so into variants/<name>/ (git-ignored; they travel to the
# GPU box with the snapshot). Usage: tools/build_variants.sh name "DEVFLAGS" [name "DEVFLAGS" ...]
# Select one at run time with PT_LIB=variants/<name>/libptamd.so.  The flags are ADDED to the product's device
# flags (the Makefile's DEVFLAGS default), so that a variant differs from the product only by what it names.
set -e
ROOT=$(cd "$(dirname "$0")/.." && pwd)
while [ $# -ge 2 ]; do
  d=$ROOT/variants/$1
  mkdir -p $d/build
  base=$(make -s -C $ROOT/cudapathtracer_amd/csrc print-devflags)
  make -s -C $ROOT/cudapathtracer_amd/csrc -j8 OUT=$d/libptamd.so OBJDIR=$d/build/ DEVFLAGS="$base $2"
  echo "built $d/libptamd.so ($2)"
  shift 2
done
