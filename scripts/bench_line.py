"""One summary line of a bench.py JSON output: name, GiB/s, reference digest match, compress / decompress GiB/s,
mismatches and the kernels above 0.5 ms per step.  usage: python scripts/bench_line.py FILE NAME"""
import json
import sys

d = json.load(open(sys.argv[1]))
ks = d["roofline"]["kernel_ms_per_step"]
print(sys.argv[2], round(d["value"], 3), (d.get("fullsize_parity") or {}).get("match"), round(d["compress_gib_s"], 3),
      round(d["decompress_gib_s"], 3), d["mismatches"], {k.split("::")[1][:24]: round(v, 1) for k, v in ks.items() if v > 0.5})
