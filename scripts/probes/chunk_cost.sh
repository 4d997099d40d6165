#!/bin/bash
# Cost of posting a message as several RCCL ops instead of one (VERDICT r2
# item 1d), on the self path of one MI355X: 256 MiB and 1 GiB messages as one
# op (P2P_RCCL_MAX_CHUNK=1G, under the 16 MiB x 64 channel limit) against
# 32 MiB ops, at 1 and 4 communicators, every delivery verified.  Prints one
# summary line per row; the JSON files stay in the output directory.
#   bash scripts/probes/chunk_cost.sh [out_dir]
set -u
OUT=${1:-gpurun_out/chunk_cost}
mkdir -p "$OUT"
for comms in 1 4; do
  for chunk in 1G 32M; do
    js="$OUT/k${comms}_${chunk}.json"
    P2P_RCCL_MAX_CHUNK=$chunk timeout -k 10 120 ./build/p2p_matrix --mode self --sizes 256M,1G -n 16 --verify \
      --comms "$comms" --no-compat --json "$js" > "$OUT/k${comms}_${chunk}.txt" 2>&1
    rc=$?
    echo "comms=$comms chunk=$chunk rc=$rc"
    if [ $rc -ne 0 ] && [ $rc -ne 2 ]; then exit $rc; fi
  done
done
python3 - "$OUT" <<'PY'
import glob, json, os, sys
out = sys.argv[1]
rows = {}
for path in sorted(glob.glob(os.path.join(out, "k*_*.json"))):
    name = os.path.basename(path)[:-5]
    for line in open(path):
        r = json.loads(line)
        if r.get("type") == "run":
            ph = r["phases"][0]
            rows[(name, r["bytes"])] = (r["gbs_mean"], ph["op_bytes"], ph["mismatches"], r["verify_coverage"])
with open(os.path.join(out, "summary.txt"), "w") as f:
    for (name, b), (gbs, op, bad, cov) in sorted(rows.items()):
        line = "%-8s %5d MiB  %8.1f GB/s  op %4d MiB  mismatches %d  coverage %s" % (name, b >> 20, gbs, op >> 20, bad, cov)
        print(line)
        f.write(line + "\n")
PY
