import re, sys
cur = None; stats = {}; order = []
for line in open(sys.argv[1]):
    m = re.match(r'^(\.LBB\w+|_Z\w+):', line)
    if m:
        cur = m.group(1); order.append(cur); stats[cur] = {}
        continue
    m = re.match(r'^\s+([a-z_0-9]+)', line)
    if m and cur:
        op = m.group(1)
        cat = 'ds' if op.startswith('ds_') else 'valu' if op.startswith('v_') else 'salu' if op.startswith('s_') and not op.startswith('s_waitcnt') and not op.startswith('s_load') else 'wait' if op.startswith('s_waitcnt') else 'vmem' if op.startswith(('global_','buffer_')) else 'smem' if op.startswith('s_load') else 'other'
        stats[cur][cat] = stats[cur].get(cat, 0) + 1
for b in order:
    st = stats[b]
    if st.get('ds', 0) >= 10 or st.get('vmem', 0) >= 2:
        print(b, st)
