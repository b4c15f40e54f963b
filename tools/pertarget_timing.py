import sys, time; sys.path.insert(0,'/root/repo/bn-pp_amd/python')
import bnpp
from bnpp import synth
ctx=bnpp.Context(0)
m=bnpp.Model.from_dict(synth.ising_grid(12,32,seed=0))
for rep in range(2):
    t=time.perf_counter(); marg, up = bnpp.marginals(ctx, m, {}, 'mf', bnpp.F64); print('mar', rep, (time.perf_counter()-t)*1e3, up, flush=True)
