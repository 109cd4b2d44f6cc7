cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/fb
for r in 1 2; do
  for b in 2 3 4 1; do
    PMC_FRONT_BATCH=$b timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/fb/b${b}_$r.json 2> gpurun_out/fb/b${b}_$r.err || exit $?
    python3 -c "import json; d=json.load(open('gpurun_out/fb/b${b}_$r.json')); print('batch $b run $r', round(d['value'],3), round(d['roofline']['kernel_ms_per_step']['pmc::deflate_front_kernel'],1))"
  done
done
