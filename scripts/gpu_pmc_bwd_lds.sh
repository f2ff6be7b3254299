# LDS bank-conflict attribution in the fused d = 64 backward (C3, non-causal): one PMC pass of
# the LDS counters per library, the product and timing-only ablations (scripts/build_abl.sh
# fa_bwd_fused BWDABL 1 4 8 32: no dQ strips, a third fewer strip reads, half the dV/dK
# transposed reads, no staging)
set -e
mkdir -p gpurun_out
export TMPDIR=/tmp
D=llmsys-project-flashattn_amd/minitorch/_lib
for lib in $D/libminitorch_hip.so $D/diag/abl_fa_bwd_fused_1.so $D/diag/abl_fa_bwd_fused_4.so $D/diag/abl_fa_bwd_fused_8.so $D/diag/abl_fa_bwd_fused_32.so; do
  t=$(basename $lib .so)
  MT_HIP_LIB=$lib ROUNDS=1 timeout -k 10 -s KILL 120 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_INSTS_MFMA --kernel-trace --kernel-include-regex fa_bwd_fused -d gpurun_out/pmcl_$t -o run --output-format csv -- python3 scripts/ablate_bwd.py 0 > gpurun_out/pmcl_$t.log 2>&1
done
python3 - <<'PY'
import csv, glob
for d in sorted(glob.glob('gpurun_out/pmcl_*/')):
    f = glob.glob(d + '*counter_collection.csv')
    if not f:
        print(d, 'no counters'); continue
    rows = list(csv.DictReader(open(f[0])))
    agg = {}
    n = len({r['Dispatch_Id'] for r in rows})
    for r in rows:
        agg[r['Counter_Name']] = agg.get(r['Counter_Name'], 0.0) + float(r['Counter_Value'])
    print(d, 'dispatches', n, {k: round(v / n) for k, v in agg.items()},
          'conflict/active', round(agg.get('SQ_LDS_BANK_CONFLICT', 0) / max(1, agg.get('SQ_LDS_IDX_ACTIVE', 1)), 4),
          'lds/mfma', round(agg.get('SQ_INSTS_LDS', 0) / max(1, agg.get('SQ_INSTS_MFMA', 1)), 3))
PY
