import sys, collections; sys.path.insert(0,'.')
import numpy as np
from tests.test_infomap import karate, codelength
import fastconsensus_amd as fc
n,e=karate()
for T in (1,10):
    with fc.Engine(seed=5) as eng:
        eng.set_option("infomap_trials", T)
        eng.load_graph(n, e[:,0], e[:,1]); eng.cd(4,0,40,40,0); lab=eng.get_labels(40)
    print("trials",T, collections.Counter([round(codelength(n,e,x),4) for x in lab]))
