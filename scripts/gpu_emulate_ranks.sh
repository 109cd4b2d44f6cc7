#!/bin/bash
# Every rank's share of N = 2/4/8 on one GPU (bench.py --emulate RANK/WORLD), checked against that rank's
# reference digests (records and member bytes).  RANKS narrows the list.
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/${TAG:-r6emu}
mkdir -p $O
for e in ${RANKS:-0/2 1/2 0/4 1/4 2/4 3/4 0/8 1/8 2/8 3/8 4/8 5/8 6/8 7/8}; do
  f=$O/rank_$(echo $e | tr / _).json
  timeout -k 10 300 python bench.py --emulate $e --no-cpu-baseline --steps 1 --warmup 1 > $f 2> $f.err || exit 1
  python3 -c "import json,sys;d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]);p=d['fullsize_parity'];print(p.get('emulated'),round(d['value'],2),p['match'],p.get('bytes_match'))" $f
done
