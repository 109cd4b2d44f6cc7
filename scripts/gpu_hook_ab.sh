#!/bin/bash
# A B A B of the f1 hook (ref_server_batch) with two builds of the drop-in: B = the tree's, A = build/ab_old
# (LD_LIBRARY_PATH wins over the binaries' RUNPATH).  SHAPES as scripts/ref_server_bench.sh.
#   /usr/local/graft/bin/gpurun -- bash scripts/gpu_hook_ab.sh
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/${TAG:-r6hookbuf}
for k in 1 2; do
  for v in old new; do
    if [ $v = old ]; then export LD_LIBRARY_PATH=$PWD/build/ab_old${LD_LIBRARY_PATH:+:$LD_LIBRARY_PATH}; fi
    OUT=$O/${v}_$k SERVERS="ref_batch" SHAPES="${SHAPES:-4096 64 65536 100000
1024 16 8192 40000}" timeout -k 10 300 bash scripts/ref_server_bench.sh > /dev/null 2>&1
    if [ $v = old ]; then export LD_LIBRARY_PATH=${LD_LIBRARY_PATH#$PWD/build/ab_old}; export LD_LIBRARY_PATH=${LD_LIBRARY_PATH#:}; fi
    while read -r l; do echo "$v run=$k $l"; done < $O/${v}_$k/ref_server_bench.jsonl
  done
done
