import sys; sys.path.insert(0,'.')
import numpy as np
from tests.test_infomap import karate, codelength
import fastconsensus_amd as fc
n,e=karate()
deg=np.bincount(e.ravel(),minlength=n)/ (2.0*len(e))
H=float((deg*np.log2(deg)).sum())
for T in (1,3):
    with fc.Engine(seed=5) as eng:
        eng.set_option("infomap_trials", T)
        eng.load_graph(n, e[:,0], e[:,1]); eng.cd(4,0,4,4,0); lab=eng.get_labels(4)
    print("T",T,"host codelength + node entropy", [round(codelength(n,e,x)+H,6) for x in lab], flush=True)
