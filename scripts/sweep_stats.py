import csv, collections, sys
for mode in range(4):
    try:
        tr = list(csv.DictReader(open(f'gpurun_out/sweep_modes/m{mode}/run_kernel_trace.csv')))
    except Exception as e:
        print(mode, e); continue
    d = collections.defaultdict(list)
    for r in tr:
        if 'vadu_sweep' in r['Kernel_Name']:
            d[r['Grid_Size_X']].append(int(r['End_Timestamp']) - int(r['Start_Timestamp']))
    print(mode, {g: (len(v), round(sum(v) / len(v) / 1e3, 1)) for g, v in d.items()})
