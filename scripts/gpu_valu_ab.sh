#!/bin/bash
# Kernel-work check of the current build: the -m gpu suite, C4 and C2 bench lines, and the C4 PMC passes
# (instruction mix, VALU breakdown, HBM bytes) summarised per kernel.  Each GPU step has its own limit and
# the steps are chained with && (stop at the first failure).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
export TMPDIR=/tmp
tag=${TAG:-r02_valu}
TESTS=${TESTS:-tests}
pmc() {  # pmc <pass> <counters...>
  local p=$1; shift
  timeout -k 10 120 rocprofv3 --pmc "$@" --output-format csv -d gpurun_out/pmc_${tag}/p$p -o run -- \
    python3 bench.py --config C4 --cpu-frames 0 --no-timing --steps 20 --warmup 3 --worst-frames 0 ${BENCH_EXTRA} > gpurun_out/pmc_${tag}_p$p.log 2>&1
}
timeout -k 10 500 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu ${TESTS} > gpurun_out/${tag}_gpu_tests.log 2>&1 &&
timeout -k 10 200 python -u bench.py --config C4 --cpu-frames 0 --steps 50 --warmup 5 ${BENCH_EXTRA} > gpurun_out/${tag}_bench_c4.log 2>&1 &&
timeout -k 10 200 python -u bench.py --cpu-frames 0 ${BENCH_EXTRA} > gpurun_out/${tag}_bench_c2.log 2>&1 &&
pmc 1 SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SMEM SQ_WAVE_CYCLES &&
pmc 2 SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INST_CYCLES_VMEM_RD GRBM_GUI_ACTIVE &&
pmc 3 SQ_INSTS_VALU_FMA_F32 SQ_INSTS_VALU_MUL_F32 SQ_INSTS_VALU_ADD_F32 SQ_INSTS_VALU_TRANS_F32 SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_INT64 SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS &&
pmc 4 FETCH_SIZE &&
pmc 5 WRITE_SIZE
rc=$?
python3 scripts/pmc_summary.py gpurun_out/pmc_${tag} --json gpurun_out/pmc_${tag}.json > gpurun_out/pmc_${tag}.txt 2>&1
tail -2 gpurun_out/${tag}_gpu_tests.log
cut -c1-400 gpurun_out/${tag}_bench_c4.log gpurun_out/${tag}_bench_c2.log 2>/dev/null
python3 - "$tag" <<'EOF'
import json, sys
try:
    d = json.load(open(f"gpurun_out/pmc_{sys.argv[1]}.json"))
except Exception as e:
    print("no pmc", e); sys.exit(0)
for k in ("k_propagate_weigh", "k_resample", "k_resample_final"):
    r = d.get(k)
    if not r or not r.get("SQ_WAVES"):
        continue
    w = r["SQ_WAVES"]
    print(k, {c[8:] if c.startswith("SQ_INSTS") else c: round(v / w, 1) for c, v in r.items()
              if c.startswith("SQ_INSTS") or c in ("SQ_WAVE_CYCLES", "SQ_WAIT_ANY", "SQ_WAIT_INST_ANY")},
          "hbm", r.get("hbm_bytes"))
EOF
exit $rc
