#!/bin/bash
# HBM traffic of the bench's kernels from PMC counters: FETCH_SIZE and WRITE_SIZE in two
# separate rocprofv3 --pmc passes (they do not fit one pass; no tracing domains mixed in),
# then tools/pmc_traffic.py applies the gfx950 FETCH_SIZE x2 correction
# (MI355X_MICROARCH.md, HBM) and writes OUTDIR/pmc_traffic.json.
# Usage: [META="k=v ..."] tools/pmc_traffic.sh OUTDIR [bench args...]
set -e
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
OUT=$(realpath -m "$1"); shift
mkdir -p "$OUT"
export TMPDIR=/tmp
cd /tmp
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$OUT/fetch" -o pmc -- \
  python3 "$R/bench.py" "$@" > "$OUT/fetch.log" 2>&1
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$OUT/write" -o pmc -- \
  python3 "$R/bench.py" "$@" > "$OUT/write.log" 2>&1
# VALU issue: wave-instructions and durations of the same launches (a third pass)
timeout -k 10 300 rocprofv3 --pmc SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_BUSY_CYCLES --output-format csv \
  -d "$OUT/valu" -o pmc -- python3 "$R/bench.py" "$@" > "$OUT/valu.log" 2>&1
python3 "$R/tools/pmc_traffic.py" "$OUT" $META > "$OUT/pmc_traffic.json"
