"""Correctly rounded 2^(j/64), j = 0..63, and the Taylor coefficients of e^(c rs) - 1 in rs
(c = ln2/64) for cf_math.h exp_tab.  Decimal arithmetic at 50 digits; float(Decimal) rounds
correctly, so every table entry is the double nearest the exact value."""
from decimal import Decimal, getcontext

getcontext().prec = 50
LN2 = Decimal(2).ln()


def main():
    tab = [float((Decimal(j) / 64 * LN2).exp()) for j in range(64)]
    c = LN2 / 64
    coef = [c ** k / Decimal(__import__("math").factorial(k)) for k in range(1, 6)]   # a1..a5
    print("// 2^(j/64), j = 0..63 (tools/gen_exp2_table.py)")
    print("static constexpr double kExp2Tab64[64] = {")
    for i in range(0, 64, 4):
        print("    " + ", ".join(v.hex() if False else repr(v) for v in tab[i:i + 4]) + ",")
    print("};")
    print("// a_k = (ln2/64)^k / k!, k = 1..5")
    print("static constexpr double kExpTabA[5] = {" + ", ".join(repr(float(a)) for a in coef) + "};")
    print("static constexpr double kInvLn2x64 = %r;   // 64 / ln2" % float(64 / LN2))


if __name__ == "__main__":
    main()
