#!/bin/bash
# PMC instruction-mix passes of one config for the base library (ab/libpfmpe_base.so) and the in-tree one:
#   pmc_ab.sh <config> [bench args...]   -> gpurun_out/pmcab_<config>_{base,new}.json
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out; export TMPDIR=/tmp
cfg=$1; shift
for v in base new; do
  if [ $v = base ]; then export PFMPE_LIB_OVERRIDE=$PWD/ab/libpfmpe_base.so; else unset PFMPE_LIB_OVERRIDE; fi
  i=0
  for set in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SMEM SQ_WAVE_CYCLES" \
             "SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INST_CYCLES_VMEM_RD GRBM_GUI_ACTIVE" \
             "SQ_INSTS_VALU_FMA_F32 SQ_INSTS_VALU_MUL_F32 SQ_INSTS_VALU_ADD_F32 SQ_INSTS_VALU_TRANS_F32 SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_INT64 SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS"; do
    i=$((i+1))
    timeout -s KILL 120 rocprofv3 --pmc $set --output-format csv -d gpurun_out/pmcab_${cfg}_$v/p$i -o run -- python3 bench.py --config $cfg --cpu-frames 0 --no-timing --worst-frames 0 --multi-sweep none --scale-ref-steps 0 "$@" > gpurun_out/pmcab_${cfg}_${v}_p$i.log 2>&1
    rc=$?; echo "$v pass $i rc=$rc"; if [ $rc -ne 0 ]; then tail -5 gpurun_out/pmcab_${cfg}_${v}_p$i.log; exit $rc; fi
  done
  python3 scripts/pmc_summary.py gpurun_out/pmcab_${cfg}_$v --json gpurun_out/pmcab_${cfg}_$v.json > /dev/null
done
unset PFMPE_LIB_OVERRIDE
python3 - "$cfg" <<'PY'
import json, sys
cfg = sys.argv[1]
b = json.load(open(f"gpurun_out/pmcab_{cfg}_base.json")); n = json.load(open(f"gpurun_out/pmcab_{cfg}_new.json"))
keys = ["SQ_INSTS_VALU", "SQ_INSTS_SALU", "SQ_INSTS_LDS", "SQ_INSTS_VMEM_RD", "SQ_INSTS_VMEM_WR", "SQ_INSTS_VALU_FMA_F32",
        "SQ_INSTS_VALU_MUL_F32", "SQ_INSTS_VALU_ADD_F32", "SQ_INSTS_VALU_INT32", "SQ_INSTS_VALU_INT64", "SQ_INSTS_VALU_TRANS_F32",
        "SQ_WAIT_INST_LDS", "SQ_LDS_BANK_CONFLICT"]
for k in sorted(set(b) & set(n)):
    w = n[k].get("SQ_WAVES") or 1
    wb = b[k].get("SQ_WAVES") or 1
    print(k, "waves", int(w))
    for c in keys:
        if c in n[k] and c in b[k]:
            print(f"   {c:26s} per wave  base {b[k][c]/wb:9.1f}  new {n[k][c]/w:9.1f}")
    for c in ("SQ_WAIT_ANY", "SQ_ACTIVE_INST_VALU", "SQ_WAIT_INST_ANY"):
        if c in n[k] and "SQ_WAVE_CYCLES" in n[k]:
            print(f"   {c:26s} / wave cycles base {b[k][c]/max(1,b[k]['SQ_WAVE_CYCLES']):.3f}  new {n[k][c]/max(1,n[k]['SQ_WAVE_CYCLES']):.3f}")
    if "SQ_ACTIVE_INST_VALU" in n[k] and "SQ_BUSY_CYCLES" in n[k]:
        print(f"   VALU active / busy cycles base {b[k]['SQ_ACTIVE_INST_VALU']/max(1,b[k]['SQ_BUSY_CYCLES']):.3f} new {n[k]['SQ_ACTIVE_INST_VALU']/max(1,n[k]['SQ_BUSY_CYCLES']):.3f}")
PY
