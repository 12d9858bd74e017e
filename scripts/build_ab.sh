#!/bin/bash
# Build an A/B variant of libpsvo.so: the working tree's sources with the
# named files taken from git revision REV (or a variant file: path=file),
# into proud-slam_amd/lib/ab/libpsvo_NAME.so (diagnostic, not the product).
#   scripts/build_ab.sh NAME REV path/in/repo [path=altfile ...] [-- EXTRA_HIPFLAGS]
set -eu
cd "$(dirname "$0")/.."
name=$1; rev=$2; shift 2
tmp=$(mktemp -d /tmp/psvo_ab_${name}_XXXX)
mkdir -p $tmp/proud-slam_amd
cp -r include $tmp/include
cp -r proud-slam_amd/csrc $tmp/proud-slam_amd/csrc
extra=""
while [ $# -gt 0 ]; do
  if [ "$1" = "--" ]; then shift; extra="$*"; break; fi
  case "$1" in
    *=*) cp "${1#*=}" "$tmp/${1%%=*}" ;;
    *) git show "$rev:$1" > "$tmp/$1" ;;
  esac
  shift
done
make -s -C $tmp/proud-slam_amd/csrc -j8 HIPFLAGS="--offload-arch=gfx950 -O3 -fPIC -std=c++17 -munsafe-fp-atomics -Wall -Wno-unused-function -fno-gpu-rdc -I../../include $extra" > /dev/null
mkdir -p proud-slam_amd/lib/ab
cp $tmp/proud-slam_amd/lib/libpsvo.so proud-slam_amd/lib/ab/libpsvo_${name}.so
rm -rf $tmp
echo "built proud-slam_amd/lib/ab/libpsvo_${name}.so"
