"""Per-variant summary of tools/pmc_variants2.sh (render kernels only, per dispatch)."""
import csv, glob, os, statistics
for d in sorted(glob.glob('gpurun_out/pmcv/*/')):
    n = os.path.basename(d[:-1])
    if n.startswith('kt_'):
        for f in glob.glob(d + '**/*kernel_trace.csv', recursive=True):
            ds = [(int(r['End_Timestamp']) - int(r['Start_Timestamp'])) / 1e6 for r in csv.DictReader(open(f))
                  if 'render_kernel' in r['Kernel_Name'] and '<true' not in r['Kernel_Name']]
            print(n, 'render dispatches (ms)', [round(x, 2) for x in ds])
        continue
    acc = {}
    for f in glob.glob(d + '**/*counter_collection.csv', recursive=True):
        for r in csv.DictReader(open(f)):
            k = r['Kernel_Name']
            if 'render_kernel' in k and '<true' not in k:
                acc.setdefault(r['Counter_Name'], {}).setdefault(r['Dispatch_Id'], 0.0)
                acc[r['Counter_Name']][r['Dispatch_Id']] += float(r['Counter_Value'])
    print(n, {c: '%.3e' % statistics.mean(v.values()) for c, v in sorted(acc.items())})
