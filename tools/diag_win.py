import sys, numpy as np
sys.path.insert(0, '.'); sys.path.insert(0, 'oracle')
import simplex_method_gpu_amd as spx, oracle
m, n, seed = 300, 1200, 7
A, b, c = oracle.generate(m, n, seed)
def rel(a, b): return float(np.max(np.abs(a-b))/max(1, np.max(np.abs(b))))
for w in (-1, 16):
    with spx.Context(A, b, c, window=w) as ctx:
        tot = 0
        for k in (13, 1, 2, 40, 44):
            ctx.iterate(k); tot += k
            s = ctx.state(binv=True)
            ref = oracle.solve(A, b, c, max_iter=tot, want_state=True)
            print(w, tot, 'binv', rel(s['binv'], ref.binv), 'xb', rel(s['x_b'], ref.x_b), 'y', rel(s['y'], ref.y), 'binv00', s['binv'][0,:3], ref.binv[0,:3])
            s2 = ctx.state(binv=True)
            print('   second state binv', rel(s2['binv'], ref.binv))
            ctx.reduced_costs()
