"""Correctly rounded 2^(j/N), j = 0..N-1 (N = 64, 256 or 1024), and the Taylor coefficients of e^(c rs) - 1 in rs
(c = ln2/N) for cf_math.h exp_tab.  Decimal arithmetic at 50 digits; float(Decimal) rounds
correctly, so every table entry is the double nearest the exact value."""
from decimal import Decimal, getcontext

getcontext().prec = 50
LN2 = Decimal(2).ln()


def main():
    import sys
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 64          # 64 (degree 5), 256 (degree 4), 1024 (degree 3)
    deg = {64: 5, 256: 4, 1024: 3}[n]
    tab = [float((Decimal(j) / n * LN2).exp()) for j in range(n)]
    c = LN2 / n
    coef = [c ** k / Decimal(__import__("math").factorial(k)) for k in range(1, deg + 1)]
    sfx = "" if n == 64 else str(n)
    print("// 2^(j/%d), j = 0..%d (tools/gen_exp2_table.py %d)" % (n, n - 1, n))
    print("static constexpr double kExp2Tab%d[%d] = {" % (n, n))
    for i in range(0, n, 4):
        print("    " + ", ".join(repr(v) for v in tab[i:i + 4]) + ",")
    print("};")
    print("// a_k = (ln2/%d)^k / k!, k = 1..%d" % (n, deg))
    print("static constexpr double kExpTabA%s[%d] = {" % (sfx, deg) + ", ".join(repr(float(a)) for a in coef) + "};")
    print("static constexpr double kInvLn2x%d = %r;   // %d / ln2" % (n, float(n / LN2), n))


if __name__ == "__main__":
    main()
