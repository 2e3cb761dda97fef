#!/bin/bash
# Build the library of git revision REV (default HEAD: the committed tree, without the
# working tree's edits) into ab/lib<TAG>.so for interleaved A/B runs (tools/ab.sh).
#   bash tools/ab_build.sh <tag> [rev] [-DDEFINE ...]
set -euo pipefail
TAG=$1; REV=${2:-HEAD}; shift; [ $# -gt 0 ] && shift
ROOT=$(cd "$(dirname "$0")/.." && pwd)
WT=$ROOT/.abtree/$TAG
rm -rf "$WT"; git -C "$ROOT" worktree prune
git -C "$ROOT" worktree add --detach -f "$WT" "$REV" >/dev/null
DEFS=$(printf "'%s'," "${@#-D}")
(cd "$WT" && python3 -c "import sys; sys.path.insert(0,'.'); from ffm_amd.build import build; print(build(out='$ROOT/ab/lib$TAG.so', defines=[${DEFS%,}] if '$*' else []))")
git -C "$ROOT" worktree remove --force "$WT"
