#!/bin/bash
# Build the library of a git revision (default HEAD) into tools/_alt/<name>.so for A/B timing
# against the working tree (tools/ab_xcd.sh).   bash tools/build_head.sh [rev] [name]
set -e
cd "$(dirname "$0")/.."
rev=${1:-HEAD}; name=${2:-a_head}
src=tools/_alt/src_$name
rm -rf "$src"; mkdir -p "$src"
git archive "$rev" wavernn_amd include | tar -x -C "$src"
(cd "$src" && python -c "import sys; sys.path.insert(0, '.'); from wavernn_amd import build as b; b.build(verbose=False)" > /dev/null 2>&1)
cp "$src/wavernn_amd/_lib/libwavernn_amd.so" "tools/_alt/$name.so"
rm -rf "$src"
echo "tools/_alt/$name.so"
