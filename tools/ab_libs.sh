#!/bin/bash
# Same-box A/B of two libpamg builds (the in-tree one = "new", $1 = a library under gpurun_ab/)
# on the level-0/1 row kernels: kbench runs alternate new, old, new, old; one JSON line per
# measurement with "lib" set. Box-to-box spread (~±4 %) is larger than most kernel changes, so
# only same-box comparisons are used to accept them.
#
#   gpurun -- 'bash tools/ab_libs.sh gpurun_ab/libpamg_prev.so gpurun_out/ab.jsonl'
set -euo pipefail
export TMPDIR=/tmp
OLD=$1
OUT=${2:-gpurun_out/ab.jsonl}
MATS=${MATS:-A0,R0,P0,A1}
mkdir -p "$(dirname "$OUT")"
: > "$OUT"
for v in new old new old; do
    if [ "$v" = old ]; then export PAMG_LIB=$OLD; else unset PAMG_LIB; fi
    timeout -k 10 200 python3 -u tools/kbench.py --n 512 --levels 2 --mats "$MATS" --ops 0,1,2,3 --reps 10 \
        --configs 1024 2>/dev/null | sed "s/^{/{\"lib\": \"$v\", /" >> "$OUT"
    echo "$v done"
done
python3 - "$OUT" <<'PY'
import collections, json, sys
d = collections.defaultdict(lambda: collections.defaultdict(list))
for l in open(sys.argv[1]):
    r = json.loads(l)
    d[(r["mat"], r["op"])][r["lib"]].append(r["ms"])
for k, v in d.items():
    print(k, "new", v["new"], "old", v["old"], "%+.1f%%" % (100 * (min(v["new"]) / min(v["old"]) - 1)))
PY
