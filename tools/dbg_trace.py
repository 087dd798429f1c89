import json, os, sys
sys.path.insert(0, 'tla-raft_amd'); sys.path.insert(0, 'tests'); sys.path.insert(0, 'oracle')
import raftmc
L = json.load(open('tests/golden/levels.json')); T = json.load(open('tests/golden/traces.json'))
for name in ['seeded_n3_v1_e2_r3', 'seeded_n3_v2_e2_r3']:
    g = L[name]; t = T[name]
    print(name, 'expected keys', [e['key'] for e in t['steps']])
    for dl in (0, 1):
        mc = raftmc.ModelChecker(raftmc.ModelConfig(n_servers=g['n'], n_vals=g['V'], max_election=g['E'], max_restart=g['R'],
             invariants=tuple(g['invariants']), spec_variant=raftmc.SPEC_SEEDED, device_levels=dl))
        res = mc.run()
        tr = mc.trace()
        print(' dl', dl, res.status, res.generated, res.distinct, res.trace_len, [list(k) if k else None for k, _ in tr])
        print('   last state equal:', tr[-1][1] == t['steps'][-1]['state'])
        mc.close()
