#!/bin/bash
# builds libspg of a git revision (default HEAD) into spartan-parallel_amd/lib/libspg_base.so, for ab_lib.sh
set -e
REV=${1:-HEAD}
R=$(cd "$(dirname "$0")/.." && pwd)
T=$(mktemp -d /tmp/spg_base.XXXX)
git -C "$R" archive "$REV" | tar -x -C "$T"
make -C "$T/spartan-parallel_amd" -j8 lib/libspg.so > "$T/build.log" 2>&1
cp "$T/spartan-parallel_amd/lib/libspg.so" "$R/spartan-parallel_amd/lib/libspg_base.so"
rm -rf "$T"
echo "built $REV -> spartan-parallel_amd/lib/libspg_base.so"
