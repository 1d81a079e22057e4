# Near-minimax coefficients of g(r) = (e^r - 1 - r)/r^2 on |r| <= ln2/2 for cf_math.h exp_poly
# (Chebyshev interpolation in 50-digit arithmetic), with the max relative error of e^r = 1 + r + r^2 g(r)
# evaluated in double Horner.  Prints: total degree, fit error, evaluated error, coefficients (r^9 first).
import mpmath as mp, numpy as np
mp.mp.dps = 50
a = mp.log(2)/2
def g(r):
    if abs(r) < mp.mpf('1e-20'): return mp.mpf(1)/2 + r/6
    return (mp.exp(r) - 1 - r)/r**2
for deg in (8, 9):
    poly, err = mp.chebyfit(g, [-a*1.0001, a*1.0001], deg+1, error=True)
    c = [float(x) for x in poly]   # highest degree first
    # evaluate e^r = 1 + r + r^2 g(r) in double Horner like the device: p=c0; p=fma(p,r,ci); p=fma(p,r,1); p=fma(p,r,1)
    xs = np.linspace(-float(a), float(a), 200001)
    worst = 0
    for x in xs[::50]:
        p = c[0]
        for ci in c[1:]: p = p*x + ci
        p = p*x + 1.0; p = p*x + 1.0
        ex = mp.exp(mp.mpf(x))
        worst = max(worst, abs(float((mp.mpf(p) - ex)/ex)))
    print(deg+2, float(err), worst, [repr(v) for v in c])
