#!/bin/bash
# Builds the library of a git revision (default HEAD) into
# find-tfbs_amd/lib/probe<NAME>/ for same-box A/B runs (tools/exp.sh NAME),
# from a temporary worktree so the working tree is untouched.
# Usage: bash tools/build_ref_lib.sh [REV] [NAME]
set -e
cd "$(dirname "$0")/.."
REV=${1:-HEAD}; NAME=${2:-prev}
WT=$(mktemp -d /tmp/tfbs_wt.XXXXXX)
git worktree add -q --detach $WT $REV
make -s -C $WT -j8 find-tfbs_amd/lib/libtfbs_amd.so > /dev/null
mkdir -p find-tfbs_amd/lib/probe$NAME
cp $WT/find-tfbs_amd/lib/libtfbs_amd.so find-tfbs_amd/lib/probe$NAME/
git worktree remove --force $WT
echo "built $REV -> find-tfbs_amd/lib/probe$NAME/libtfbs_amd.so"
