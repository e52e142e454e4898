#!/bin/bash
# Build an alternate engine library for A/B runs (tools/ab_run.py loads it in place of the tree's).
#   bash tools/build_variant.sh <tag> [git-rev|-] [extra hipcc flags...]
# rev "-" (default) builds the working tree's sources; a git rev builds that commit's.
# Output: tools/ab/libsgx_<tag>.so (git-ignored, travels to the GPU box with the snapshot).
set -e
tag=$1; rev=${2:--}; shift; [ $# -gt 0 ] && shift
root=$(cd "$(dirname "$0")/.." && pwd)
work=/tmp/sgx_variant_$tag
rm -rf "$work"; mkdir -p "$work"
if [ "$rev" = "-" ]; then
  cp -r "$root/sparkucx_amd" "$root/include" "$work/"
else
  git -C "$root" archive "$rev" sparkucx_amd/csrc include | tar -x -C "$work"
fi
make -s -C "$work/sparkucx_amd/csrc" -j8 OUT="$root/tools/ab/libsgx_$tag.so" \
  HIPFLAGS="-O3 -std=c++17 -fPIC --offload-arch=gfx950 -Wall -Wno-unused-result -munsafe-fp-atomics $*"
echo "built tools/ab/libsgx_$tag.so"
