#!/bin/bash
# Build an A/B variant of libnerfmi.so from patched sources (nothing in the tree changes):
#   scripts/build_variant.sh NAME 'python-replacement-expr'
# copies the package to /tmp/var_NAME, runs the python snippet there (it edits csrc/ files), builds,
# and copies the library to depth-aware-shader-effects-for-nerf_amd/build/ab/libnerfmi_NAME.so.
set -e
NAME=$1; PATCH=$2
ROOT=$(cd "$(dirname "$0")/.." && pwd)
rm -rf /tmp/var_$NAME && mkdir -p /tmp/var_$NAME
cp -r "$ROOT/depth-aware-shader-effects-for-nerf_amd" /tmp/var_$NAME/pkg
cp -r "$ROOT/include" /tmp/var_$NAME/include
cd /tmp/var_$NAME/pkg && rm -rf build libnerfmi.so
python3 -c "$PATCH"
make -j8 libnerfmi.so > /tmp/var_$NAME/build.log 2>&1 || { tail -20 /tmp/var_$NAME/build.log; exit 1; }
mkdir -p "$ROOT/depth-aware-shader-effects-for-nerf_amd/build/ab"
cp libnerfmi.so "$ROOT/depth-aware-shader-effects-for-nerf_amd/build/ab/libnerfmi_$NAME.so"
echo "built build/ab/libnerfmi_$NAME.so"
