#!/bin/bash
set -o pipefail
S8=6144x4096,4096x4096,28672x4096,4096x14336
for cfg in "0 768 2" "1 1536 8" "1 1536 4"; do set -- $cfg
  OGKM_DGEMM_LDS=$1 OGKM_DGEMM_UNITS=$2 SHAPES=$S8 VARIANTS=raw:$3 timeout -k 10 120 python -u tools/bench_dgemm.py 2>&1 | grep '^{' | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('8b lds=$1 units=$2 u=$3', d['per_shape_ms'])"
  OGKM_DGEMM_LDS=$1 OGKM_DGEMM_UNITS=$2 VARIANTS=raw:$3 timeout -k 10 120 python -u tools/bench_dgemm.py 2>&1 | grep '^{' | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('70b lds=$1 units=$2 u=$3', d['per_shape_ms'])"
done
