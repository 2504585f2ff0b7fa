import json,glob,sys
for f in sorted(glob.glob('gpurun_out/ab/*.json')):
    try: d=json.loads(open(f).read().strip().splitlines()[-1])
    except Exception as e: print(f, 'ERR', e); continue
    if 'c2' not in d: continue
    print(f, 'c4', round(d['value']), 'c2', round(d['c2']['value']), 'c3s', round(d['c3']['single_pair']['value']), 'c3b', round(d['c3']['batch']['value']), 'c5s', round(d['c5']['streamed']['value']), 'c2err', d['c2']['pose_max_abs_err_vs_cpu'])
