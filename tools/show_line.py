"""Print the main fields of bench.py JSON lines (files given on the command line)."""
import json
import sys

for f in sys.argv[1:]:
    try:
        d = json.loads(open(f).read().strip().splitlines()[-1])
    except Exception as e:  # noqa: BLE001
        print(f, e)
        continue
    keys = ['value', 'ms_per_step', 'scaling', 'train_steps_per_s', 'cifar_train_steps_per_s',
            'pinn_train_steps_per_s', 'dps_nfe_per_s', 'ns_gsites_per_s', 'ncddpmpp_evals_per_s']
    print(f, {k: d.get(k) for k in keys if d.get(k) is not None})
    r = d.get('roofline')
    if r:
        print('  roof', r['frac'], r['ms_per_mix'], [(p['shape'], p['pre_tflops']) for p in r['per_shape']])
    for k in ('roofline_train', 'roofline_cifar_train', 'roofline_pinn', 'roofline_dps'):
        if d.get(k):
            print('  ', k, d[k]['frac'])
    u = d.get('roofline_upfirdn2d')
    if u:
        print('  upfirdn', [(x['kernel'][9:30], x['frac'], x['traffic']) for x in u])
    if d.get('cpu_baseline'):
        print('  cpu', d['cpu_baseline']['value'], {k: v.get('value') for k, v in d.get('cpu_baselines_other', {}).items()})
