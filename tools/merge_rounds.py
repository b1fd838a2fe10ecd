import sys, time; sys.path.insert(0,'/root/repo')
import uno_amd, numpy as np
n,nv,m,r,c,v,b = uno_amd.arrowband(int(sys.argv[1]), uno_amd.SEEDS["C3"])
g=uno_amd.HipKKT(0); g.set_option("verbose",1)
t=time.time(); g.analyze(n,r,c); print("analyze", time.time()-t, flush=True)
t=time.time(); g.factorize(v); print(g.inertia(), "first factorization", time.time()-t, flush=True)
t=time.time(); g.factorize(v); print(g.inertia(), "second", time.time()-t, flush=True)
v2=v.copy(); v2[:nv]+=1e-4
t=time.time(); g.factorize(v2); print(g.inertia(), "regularized", time.time()-t, flush=True)
