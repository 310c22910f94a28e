import numpy as np, sys
a=np.load(sys.argv[1]); b=np.load(sys.argv[2])
for k in a.files:
    print(k, 'bitwise equal' if np.array_equal(a[k], b[k]) else 'DIFFER max %g' % np.abs(a[k].astype(np.float64)-b[k]).max())
