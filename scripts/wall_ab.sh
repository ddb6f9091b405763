#!/bin/bash
# Two-lane wall time of gg_precluster_files calls (scripts/ingest_ab.py, one
# setting per process: knobs read once per process, or an alternate build as
# GALAHGPU_LIB) on C2-like files, settings interleaved over ROUNDS rounds.
#   scripts/wall_ab.sh FILES CALLS ROUNDS 'name:K=V,K=V' ...
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
n=$1; calls=$2; rounds=$3; shift 3
for r in $(seq 1 $rounds); do
  for spec in "$@"; do
    name=${spec%%:*}; kv=${spec#*:}
    (
      IFS=',' read -ra pairs <<< "$kv"
      for p in "${pairs[@]}"; do [ -n "$p" ] && export "$p"; done
      timeout -k 10 200 python3 -u scripts/ingest_ab.py $n $calls "$name:" | grep setting
    ) || exit 1
  done
done
