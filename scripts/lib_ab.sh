#!/bin/bash
# Device-inflate timing of alternate library builds (scripts/ab_lib.sh), one
# process per build, each as scripts/ingest_ab.py reports it; the HEAD build
# first and last.  usage: scripts/lib_ab.sh FILES CALLS name [name ...]
cd "$(dirname "$0")/.."
files=$1; calls=$2; shift 2
run() {  # name lib
  if [ -n "$2" ]; then GALAHGPU_LIB=$2 timeout -k 10 240 python -u scripts/ingest_ab.py $files $calls "$1:" | grep setting
  else timeout -k 10 240 python -u scripts/ingest_ab.py $files $calls "$1:" | grep setting; fi
}
run head "" || exit 1
for n in "$@"; do run $n galah_amd/lib/ab/libgalahgpu_$n.so || exit 1; done
run head2 ""
