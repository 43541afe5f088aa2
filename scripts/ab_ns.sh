#!/bin/bash
# Interleaved A/B of the NS training step: bench.py --config ns with the in-tree library
# ("cur") and abl/abl_<name>.so variants. usage: scripts/ab_ns.sh name1 [name2 ...]
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/ab_ns
for rep in 1 2; do
  for v in cur "$@"; do
    if [ "$v" = cur ]; then L=; else L=abl/abl_$v.so; fi
    MMRE_LIB=$L timeout -k 10 200 python -u bench.py --config ns --no-cpu-baseline \
        > gpurun_out/ab_ns/$v.$rep.json 2> gpurun_out/ab_ns/$v.$rep.err || exit 1
    python - "$v" gpurun_out/ab_ns/$v.$rep.json <<'PY'
import json, sys
d = [json.loads(l) for l in open(sys.argv[2]) if l.startswith("{")][0]
print(sys.argv[1], "step_ms %.4f" % d["ms_per_step"], "fused_ms %.4f" % d["roofline"]["kernel_ms"], d["build"]["sha256"])
PY
  done
done
