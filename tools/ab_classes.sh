#!/bin/bash
# Same-box A/B of library builds with the in-step kernel classes (bench.py's kernel-trace probe) per build:
#   tools/ab_classes.sh TAG "bench args" lib1 lib2 ...   (lib = a directory under clip-ebc_amd/lib, "." = the default)
# -> gpurun_out/TAG_<lib>_r<round>.json per run and a summary table gpurun_out/TAG_classes.txt
set -o pipefail
TAG=$1; ARGS=$2; shift 2
O=gpurun_out; mkdir -p $O
for r in 1 2; do
  for l in "$@"; do
    n=$(echo "$l" | tr './' '_d')
    timeout -k 10 300 env EBC_LIB_PATH=clip-ebc_amd/lib/$l/libebc_hip.so python -u bench.py $ARGS --no-cpu-baseline \
      > $O/${TAG}_last.log 2>&1 || { echo "FAILED $l"; tail -20 $O/${TAG}_last.log; exit 1; }
    tail -1 $O/${TAG}_last.log > $O/${TAG}_${n}_r$r.json
    python -c "import json; d=json.load(open('$O/${TAG}_${n}_r$r.json')); print('$l r$r', d['value'], d['median_ms_per_step'])"
  done
done
python - "$TAG" "$@" > $O/${TAG}_classes.txt <<'EOF'
import json, sys
tag, libs = sys.argv[1], sys.argv[2:]
runs = {}
for l in libs:
    n = l.replace('.', '_').replace('/', 'd')
    runs[l] = [json.load(open(f"gpurun_out/{tag}_{n}_r{r}.json")) for r in (1, 2)]
keys = []
for l in libs:
    for d in runs[l]:
        for k in d.get("kernels", []):
            if k["kernel"] not in keys:
                keys.append(k["kernel"])
print(f"{'class (per-step us, mean of 2 runs)':60s}" + "".join(f"{l:>12s}" for l in libs))
print(f"{'crops/s':60s}" + "".join(f"{sum(d['value'] for d in runs[l]) / 2:12.1f}" for l in libs))
print(f"{'median ms/step':60s}" + "".join(f"{sum(d['median_ms_per_step'] for d in runs[l]) / 2:12.4f}" for l in libs))
for k in keys:
    row = []
    for l in libs:
        v = [x["per_step_us"] for d in runs[l] for x in d.get("kernels", []) if x["kernel"] == k]
        row.append(sum(v) / len(v) if v else float("nan"))
    print(f"{k[:60]:60s}" + "".join(f"{v:12.1f}" for v in row))
EOF
cat $O/${TAG}_classes.txt
