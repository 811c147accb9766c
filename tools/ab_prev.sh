#!/bin/bash
# Stage a git revision (default HEAD) as an A/B package variant for profiles/ab_pkg.sh:
# abpkg/<name>/VAESNe + abpkg/<name>/libvaesne_hip.so built from that revision's sources.
#   bash tools/ab_prev.sh [rev] [name]
set -e
cd "$(dirname "$0")/.."
rev=${1:-HEAD}; name=${2:-prev}
tmp=$(mktemp -d /tmp/abprev.XXXX)
git archive "$rev" vaesne-dev_amd include | tar -x -C "$tmp"
python "$tmp/vaesne-dev_amd/build_lib.py" > /dev/null
rm -rf "abpkg/$name" && mkdir -p "abpkg/$name"
cp -r "$tmp/vaesne-dev_amd/VAESNe" "abpkg/$name/VAESNe"
cp "$tmp/vaesne-dev_amd/lib/libvaesne_hip.so" "abpkg/$name/libvaesne_hip.so"
rm -rf "$tmp"
echo "abpkg/$name <- $rev"
