"""Per-kernel-shape summary of tools/gpujob_pmc_unet.sh counter passes (development tool)."""
import csv, collections, sys
data = collections.defaultdict(lambda: collections.defaultdict(float))
cnt = collections.defaultdict(lambda: collections.Counter())
dur = collections.defaultdict(dict)
pat = sys.argv[1:] or ['conv_gemm', 'attention', 'splitk', 'gn_fused']
for f in ['gpurun_out/pmc_u1/run_counter_collection.csv', 'gpurun_out/pmc_u2/run_counter_collection.csv']:
    for x in csv.DictReader(open(f)):
        kn = x['Kernel_Name']
        if not any(p in kn for p in pat):
            continue
        key = (kn[:34], int(x['Grid_Size']) // int(x['Workgroup_Size']))
        data[key][x['Counter_Name']] += float(x['Counter_Value'])
        cnt[key][x['Counter_Name']] += 1
        dur[key][(f, x['Dispatch_Id'])] = int(x['End_Timestamp']) - int(x['Start_Timestamp'])
rows = []
for k, d in data.items():
    c = cnt[k]
    g = lambda n: d[n] / max(c[n], 1)
    t = sum(dur[k].values()) / len(dur[k])
    wc = g('SQ_WAVE_CYCLES') or 1
    m = max(g('SQ_INSTS_MFMA'), 1)
    rows.append((t * c['SQ_WAVE_CYCLES'], k, round(t / 1e3, 1), c['SQ_WAVE_CYCLES'],
                 'wait %.2f instst %.2f act %.2f' % (g('SQ_WAIT_ANY') / wc, g('SQ_WAIT_INST_ANY') / wc, g('SQ_ACTIVE_INST_ANY') / wc),
                 'valu/mfma %.1f lds/mfma %.2f vmem/mfma %.2f salu/mfma %.1f conf %.2f' % (
                     g('SQ_INSTS_VALU') / m, g('SQ_INSTS_LDS') / m, g('SQ_INSTS_VMEM') / m, g('SQ_INSTS_SALU') / m,
                     g('SQ_LDS_BANK_CONFLICT') / max(g('SQ_LDS_IDX_ACTIVE'), 1))))
for r in sorted(rows, key=lambda x: -x[0])[:12]:
    print(*r[1:])
