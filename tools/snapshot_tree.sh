#!/bin/bash
# Build a runnable copy of a git revision (its Python package, bench.py and its
# own in-tree extension) under variants/<name>/ for `tools/gpu.sh ab:dir=...`
# A/B runs against the working tree.
# Usage: bash tools/snapshot_tree.sh <name> [revision, default HEAD]
set -e
ROOT=$(cd "$(dirname "$0")/.." && pwd)
NAME=$1; REV=${2:-HEAD}
WT=/tmp/mpitree_snapshot_$NAME
rm -rf "$WT"
git -C "$ROOT" worktree prune
git -C "$ROOT" worktree add -q --detach "$WT" "$REV"
(cd "$WT" && python -m mpitree_amd.ops.build > /dev/null)
rm -rf "$ROOT/variants/$NAME"
mkdir -p "$ROOT/variants/$NAME"
cp -r "$WT/mpitree_amd" "$WT/bench.py" "$ROOT/variants/$NAME/"
find "$ROOT/variants/$NAME" -name '__pycache__' -prune -exec rm -rf {} +
git -C "$ROOT" worktree remove --force "$WT"
echo "variants/$NAME ($(git -C "$ROOT" rev-parse --short "$REV"))"
