import sys; sys.path.insert(0, '.')
import numpy as np
import fastconsensus_amd as fc
e = np.array([[0, 1], [1, 2], [0, 2], [3, 4], [4, 5], [3, 5], [6, 7], [7, 8]], np.int32)
for n, store in [(12, 1), (12, 0), (9, 1), (9, 0), (5, 1)]:
    for ed in (e[e.max(1) < n], np.zeros((0, 2), np.int32)):
        try:
            with fc.Engine(seed=3) as eng:
                eng.set_option("store", store)
                eng.load_graph(n, ed[:, 0], ed[:, 1])
                print("ok", n, store, len(ed), flush=True)
        except Exception as ex:
            print("FAIL", n, store, len(ed), ex, flush=True)
