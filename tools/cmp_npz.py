import sys, numpy as np
a, b = np.load(sys.argv[1]), np.load(sys.argv[2])
for k in a.files:
    x, y = a[k], b[k]
    d = ~((x == y) | (np.isnan(x) & np.isnan(y))) if x.dtype.kind == 'f' else (x != y)
    print(k, x.shape, "differ:", int(d.sum()))
