import sys, time; sys.path[:0]=['pla-gnn_amd','.']
import numpy as np, torch
from scipy.sparse import random as sprandom
from plagnn import data, ecc
from plagnn.pca import pca
from scipy.sparse import coo_matrix
ds = data.make_dataset("s0", seed=70)
adj = coo_matrix((np.ones(len(ds.row), np.int64), (ds.row, ds.col)), shape=(ds.n, ds.n))
m = ecc.edge_clustering_coefficients(adj)
pca(m, 250); torch.cuda.synchronize()
for _ in range(2):
    t0=time.perf_counter(); f=pca(m, 250); torch.cuda.synchronize(); print("pca wall", time.perf_counter()-t0)
t0=time.perf_counter(); om=np.random.RandomState(42).normal(size=(ds.n,260)); print("omega", time.perf_counter()-t0)
