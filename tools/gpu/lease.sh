#!/bin/bash
# One GPU lease, many steps: tools/gpu/lease.sh PLAN [TAG]
#
# PLAN is a text file of steps, one per line: `name | timeout_s | command`.  Each command runs
# from the repo root under `timeout -k 10 <timeout_s>`, its output in gpurun_out/<TAG>/<name>.log
# (TAG defaults to the plan's base name).  The first failing step ends the lease (a GPU fault,
# abort or time limit must not be followed by more GPU work); its log tail is printed.  Blank
# lines and lines starting with # are skipped.  Inside a command, $O is the output directory
# and $R the repo root; rocprofv3 commands should `cd /tmp` first (TMPDIR is /tmp).
#
# This replaces the per-round one-off lease scripts (r04_*.sh, r05_*.sh): their steps are
# plans under tools/gpu/plans/.
set -o pipefail
PLAN=$1
[ -f "$PLAN" ] || { echo "usage: $0 PLAN [TAG]"; exit 64; }
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/../.." && pwd)}
TAG=${2:-$(basename "$PLAN" .txt)}
O=$R/gpurun_out/$TAG
mkdir -p "$O"
export R O TMPDIR=/tmp
cd "$R"
while IFS= read -r line || [ -n "$line" ]; do
  case "$line" in ''|'#'*) continue ;; esac
  name=$(echo "${line%%|*}" | xargs)
  rest=${line#*|}
  to=$(echo "${rest%%|*}" | xargs)
  cmd=${rest#*|}
  echo "== $name (${to}s): $cmd"
  t0=$(date +%s)
  ( cd "$R" && timeout -k 10 "$to" bash -c "$cmd" ) > "$O/$name.log" 2>&1
  st=$?
  echo "   exit $st after $(( $(date +%s) - t0 ))s"
  if [ $st -ne 0 ]; then
    tail -40 "$O/$name.log"
    exit $st
  fi
  tail -3 "$O/$name.log" | cut -c1-400
done < "$PLAN"
