#!/bin/bash
# Quick GPU parity bisection over env variants (PBFT cases through tests/parity_run.py):
#   bash tests/gpu_bisect.sh "<cases>" "<env1>" "<env2>" ...
set -o pipefail
cases=$1; shift
for v in "$@"; do
  echo "== [$v]"
  env $v timeout -k 10 200 python tests/parity_run.py $cases 2>&1 | cut -c1-220
  rc=$?; [ $rc -eq 124 -o $rc -eq 137 -o $rc -eq 3 ] && exit 1
done
exit 0
