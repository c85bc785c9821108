import json, sys
for l in open(sys.argv[1]):
    l = l.strip()
    if l.startswith('{'):
        d = json.loads(l)
        print({k: (round(v, 1) if isinstance(v, float) else v) for k, v in d.items() if k not in ('P', 'bytes', 'K')})
