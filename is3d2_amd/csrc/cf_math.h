// cf_math.h -- Cooper-Frye math shared by the HIP kernels (and, for tests only,
// by a host harness that runs the same functions serially against the oracle).
//
// The reference evaluates, for every (cell, species, pT, phi, y, eta) point, one
// exp + sinh + sqrt + 1-2 divisions (MomentumSpectra.cpp:302-361).  Here the
// integrand is factorised along the momentum grid axes:
//
//   p^tau = mT ch,  p^eta = mT sh / tau,  p^x = pT cos(phi),  p^y = pT sin(phi)
//   u.p      = mT A_q - pT B_j              A_q = ch ut - sh (tau u^eta),  B_j = cos ux + sin uy
//   p.dsigma = mT D_q + pT Dp_j             D_q = ch dat + sh dan/tau,      Dp_j = cos dax + sin day
//   pi.pp    = mT^2 Q1_q + mT pT (ch Pt_j + sh Pn_j) + pT^2 Q3_j
//   V.p      = mT W_q - pT Wp_j
//   exp(u.p/T - chem) = exp(mT A_q/T - chem) * exp(-pT B_j/T)
//
// so that the per-point work is a handful of FMAs plus one reciprocal; the
// exponentials move to per-(cell,y/eta) ("y-terms", q index) and per-(cell,phi)
// ("phi-terms", j index) tables.  For the modified distributions (PTM/PTB/PTMA)
// p_mod = A^{-1} p_LRF is linear in (mT ch, mT sh, pT cos, pT sin), so
//   p_mod = mT (ch Uc + sh Us) + pT (cos Vc + sin Vs)
// with four 3-vectors per cell (Uc = A^{-1}(-Xt,0,-Zt), Us = A^{-1}(tau Xn,0,tau Zn),
// Vc = A^{-1}(Xx,Yx,0), Vs = A^{-1}(Xy,Yy,0)).  The reference's iterative
// refinement of A p_mod = p_LRF (<=5 steps, residual 1e-16) only removes rounding
// from that same linear solve, so it is not repeated.
#pragma once
#include <math.h>

#if defined(__HIPCC__) || defined(__HIP__)
#define IS3D_HD __host__ __device__ inline
#else
#define IS3D_HD inline
#endif

namespace is3d {

// exp(x) for |x| <= 690 (the fast-path domain: no overflow, no subnormal result).
// Reduction x = k ln2 + r with k = rint(x log2 e) taken from the low word of x log2 e + 1.5 2^52
// (one FMA gives both k as a double and k as an int, no conversion), Cody-Waite r in two FMAs,
// e^r = 1 + r + r^2 g(r) with g a degree-9 near-minimax (Chebyshev) fit on |r| <= ln2/2
// (tools/fit_exp.py; 1.5e-16 relative measured in double Horner), 2^k by ldexp: 16 VALU ops,
// max error ~1 ulp against glibc (test_kernel_math_cpu).
// On the device each coefficient passes through an empty asm that pins it to an SGPR pair at
// the point of use: otherwise the compiler hoists all of them out of the cell loop into VGPRs
// and spills them to scratch (one serialized reload per coefficient per lane setup).
IS3D_HD double kconst(double v) {
#if defined(__HIP_DEVICE_COMPILE__)
  asm volatile("" : "+s"(v));
#endif
  return v;
}

struct ExpCoef { double l2e, shift, ln2hi, ln2lo, ln2, c[10]; };   // c: g(r) coefficients, r^9 first

IS3D_HD ExpCoef exp_coef() {
  ExpCoef e;
  e.l2e = kconst(1.4426950408889634);
  e.shift = kconst(6755399441055744.0);                  // 1.5 * 2^52
  e.ln2hi = kconst(6.93147180369123816490e-01);    // low 32 bits zero
  e.ln2lo = kconst(1.90821492927058770002e-10);
  e.ln2 = kconst(6.93147180559945286227e-01);
  const double f[10] = {2.510038549551032e-08, 2.7620088445409746e-07, 2.7557268459997064e-06,
                        2.4801521295954376e-05, 0.00019841269863053618, 0.0013888888917213717,
                        0.008333333333330062, 0.04166666666662413, 0.16666666666666669, 0.5000000000000001};
  for (int i = 0; i < 10; i++) e.c[i] = kconst(f[i]);
  return e;
}

// valid for |x| < 2^30 (k must fit the low word); exp_clamped handles everything else
IS3D_HD double exp_poly(const ExpCoef& E, double x) {
  const double t = fma(x, E.l2e, E.shift);
  const double k = t - E.shift;
  double r = fma(-k, E.ln2hi, x);
  r = fma(-k, E.ln2lo, r);
  double p = E.c[0];
  for (int i = 1; i < 10; i++) p = fma(p, r, E.c[i]);
  p = fma(p, r, 1.0);
  p = fma(p, r, 1.0);
  return ldexp(p, (int)(unsigned)__builtin_bit_cast(unsigned long long, t));
}

// As exp_poly with a one-FMA reduction r = x - k ln2 (k ln2 exact inside the FMA; the error
// |k| |ln2 - ln2_double| <= |k| 2.3e-17 is a third of the rounding error |x| 2^-53 >= |k| 7.7e-17
// that any double argument x already carries, so the result's accuracy relative to the exact
// exp of the exact argument is unchanged).  Used per point on the modified-momentum path.
IS3D_HD double exp_poly1(const ExpCoef& E, double x) {
  const double t = fma(x, E.l2e, E.shift);
  const double k = t - E.shift;
  const double r = fma(-k, E.ln2, x);
  double p = E.c[0];
  for (int i = 1; i < 10; i++) p = fma(p, r, E.c[i]);
  p = fma(p, r, 1.0);
  p = fma(p, r, 1.0);
  return ldexp(p, (int)(unsigned)__builtin_bit_cast(unsigned long long, t));
}

IS3D_HD double exp_dom690(double x) { return exp_poly(exp_coef(), x); }

// Table-driven exp for the per-point exponentials of the modified-momentum path, taking
// xN = x N/ln2 (the caller folds N/ln2 into its coefficients; N = kExpTabN = 256 by default, 64 as
// the alternative build): K = rint(xN) from the low word of xN + 1.5 2^52, rs = xN - K (exact),
// e^x = 2^(K / N) 2^((K mod N)/N) e^(c rs) with c = ln2/N, e^(c rs) - 1 = rs (a1 + rs (a2 + ...))
// (Taylor through degree 4 for N = 256, 5 for N = 64: |c rs| <= ln2/(2N) leaves < 4e-17 truncation),
// and T = 2^((K mod N)/N) correctly rounded from an N-entry table the kernels keep in LDS:
// 8 FP64 + 3 INT32 ops (N = 256) instead of exp_poly1's 15 FP64, ~1 ulp.  The error of xN itself
// (~|x| 2e-16 absolute in x) is the same order as the rounding of the exponent argument that the
// reference's own exp(E/T - chem) carries.  Valid for |xN| < 2^50; underflow / overflow via ldexp.
// 2^(j/64), j = 0..63 (tools/gen_exp2_table.py)
static constexpr double kExp2Tab64[64] = {
    1.0, 1.0108892860517005, 1.0218971486541166, 1.0330248790212284,
    1.0442737824274138, 1.0556451783605572, 1.0671404006768237, 1.0787607977571199,
    1.0905077326652577, 1.102382583307841, 1.1143867425958924, 1.1265216186082418,
    1.1387886347566916, 1.1511892299529827, 1.1637248587775775, 1.1763969916502812,
    1.189207115002721, 1.202156731452703, 1.215247359980469, 1.22848053610687,
    1.241857812073484, 1.255380757024691, 1.2690509571917332, 1.2828700160787783,
    1.2968395546510096, 1.3109612115247644, 1.3252366431597413, 1.339667524053303,
    1.3542555469368927, 1.3690024229745905, 1.383909881963832, 1.3989796725383112,
    1.4142135623730951, 1.42961333839197, 1.4451808069770467, 1.460917794180647,
    1.4768261459394993, 1.4929077282912648, 1.5091644275934228, 1.5255981507445384,
    1.5422108254079407, 1.559004400237837, 1.5759808451078865, 1.593142151342267,
    1.6104903319492543, 1.6280274218573478, 1.645755478153965, 1.6636765803267364,
    1.681792830507429, 1.7001063537185235, 1.718619298122478, 1.7373338352737062,
    1.7562521603732995, 1.7753764925265212, 1.7947090750031072, 1.8142521755003989,
    1.8340080864093424, 1.8539791250833855, 1.8741676341103, 1.8945759815869656,
    1.9152065613971474, 1.9360617934922943, 1.9571441241754002, 1.978456026387951,
};
// a_k = (ln2/64)^k / k!, k = 1..5
static constexpr double kExpTabA[5] = {0.010830424696249145, 5.86490495505617e-05, 2.1173137155464776e-07, 5.732851688640402e-10, 1.2417843701716925e-12};
static constexpr double kInvLn2x64 = 92.33248261689366;   // 64 / ln2
// 2^(j/256), j = 0..255 (tools/gen_exp2_table.py 256)
static constexpr double kExp2Tab256[256] = {
    1.0, 1.0027112750502025, 1.0054299011128027, 1.0081558981184175,
    1.0108892860517005, 1.0136300849514894, 1.016378314910953, 1.019133996077738,
    1.0218971486541166, 1.0246677928971357, 1.0274459491187637, 1.030231637686041,
    1.0330248790212284, 1.0358256936019572, 1.0386341019613787, 1.041450124688316,
    1.0442737824274138, 1.0471050958792898, 1.0499440858006872, 1.0527907730046264,
    1.0556451783605572, 1.0585073227945128, 1.061377227289262, 1.0642549128844645,
    1.0671404006768237, 1.0700337118202419, 1.0729348675259756, 1.075843889062791,
    1.0787607977571199, 1.0816856149932152, 1.0846183622133092, 1.0875590609177697,
    1.0905077326652577, 1.0934643990728858, 1.0964290818163769, 1.099401802630222,
    1.102382583307841, 1.1053714457017412, 1.1083684117236787, 1.1113735033448175,
    1.1143867425958924, 1.1174081515673693, 1.1204377524096067, 1.12347556733302,
    1.1265216186082418, 1.129575928566288, 1.1326385195987192, 1.1357094141578055,
    1.1387886347566916, 1.1418762039695616, 1.1449721444318042, 1.148076478840179,
    1.1511892299529827, 1.154310420590216, 1.1574400736337511, 1.1605782120274988,
    1.1637248587775775, 1.1668800369524817, 1.1700437696832502, 1.1732160801636373,
    1.1763969916502812, 1.1795865274628758, 1.182784710984341, 1.1859915656609938,
    1.189207115002721, 1.1924313825831512, 1.1956643920398273, 1.1989061670743806,
    1.202156731452703, 1.2054161090051239, 1.2086843236265816, 1.2119613992768012,
    1.215247359980469, 1.2185422298274085, 1.2218460329727576, 1.2251587936371455,
    1.22848053610687, 1.2318112847340759, 1.2351510639369334, 1.2384998981998165,
    1.241857812073484, 1.245224830175258, 1.2486009771892048, 1.2519862778663162,
    1.255380757024691, 1.2587844395497165, 1.2621973503942507, 1.2656195145788063,
    1.2690509571917332, 1.2724917033894028, 1.275941778396392, 1.2794012075056693,
    1.2828700160787783, 1.2863482295460256, 1.2898358734066657, 1.2933329732290895,
    1.2968395546510096, 1.3003556433796506, 1.3038812651919358, 1.3074164459346773,
    1.3109612115247644, 1.3145155879493546, 1.318079601266064, 1.3216532776031575,
    1.3252366431597413, 1.3288297242059544, 1.3324325470831615, 1.3360451382041458,
    1.339667524053303, 1.3432997311868353, 1.3469417862329458, 1.3505937158920345,
    1.3542555469368927, 1.3579273062129011, 1.3616090206382248, 1.365300717204012,
    1.3690024229745905, 1.3727141650876684, 1.3764359707545302, 1.380167867260238,
    1.383909881963832, 1.387662042298529, 1.3914243757719262, 1.3951969099662003,
    1.3989796725383112, 1.4027726912202048, 1.4065759938190154, 1.4103896082172707,
    1.4142135623730951, 1.4180478843204152, 1.4218926021691656, 1.4257477441054942,
    1.42961333839197, 1.433489413367789, 1.4373759974489824, 1.4412731191286257,
    1.4451808069770467, 1.449099089642035, 1.4530279958490526, 1.4569675544014438,
    1.460917794180647, 1.4648787441464057, 1.4688504333369818, 1.4728328908693675,
    1.4768261459394993, 1.4808302278224719, 1.4848451658727524, 1.488870989524397,
    1.4929077282912648, 1.4969554117672355, 1.5010140696264256, 1.5050837316234065,
    1.5091644275934228, 1.5132561874526098, 1.5173590411982147, 1.5214730189088146,
    1.5255981507445384, 1.529734466947287, 1.533881997840956, 1.5380407738316568,
    1.5422108254079407, 1.5463921831410214, 1.550584877685, 1.5547889397770887,
    1.559004400237837, 1.5632312899713576, 1.567469639965553, 1.5717194812923414,
    1.5759808451078865, 1.5802537626528246, 1.5845382652524937, 1.588834384317164,
    1.593142151342267, 1.597461597908627, 1.6017927556826934, 1.606135656416771,
    1.6104903319492543, 1.6148568142048607, 1.6192351351948637, 1.6236253270173289,
    1.6280274218573478, 1.632441451987275, 1.6368674497669644, 1.6413054476440063,
    1.645755478153965, 1.6502175739206177, 1.6546917676561943, 1.6591780921616162,
    1.6636765803267364, 1.6681872651305825, 1.6727101796415966, 1.6772453570178785,
    1.681792830507429, 1.6863526334483934, 1.6909247992693053, 1.6955093614893326,
    1.7001063537185235, 1.7047158096580513, 1.709337763100463, 1.713972247929926,
    1.718619298122478, 1.723278947746274, 1.7279512309618377, 1.732636182022311,
    1.7373338352737062, 1.7420442251551564, 1.746767386199169, 1.7515033530318782,
    1.7562521603732995, 1.761013843037584, 1.7657884359332727, 1.7705759740635547,
    1.7753764925265212, 1.7801900265154245, 1.785016611318935, 1.789856282321401,
    1.7947090750031072, 1.7995750249405351, 1.804454167806624, 1.809346539371032,
    1.8142521755003989, 1.8191711121586085, 1.8241033854070534, 1.8290490314048973,
    1.8340080864093424, 1.8389805867758937, 1.843966568958626, 1.8489660695104508,
    1.8539791250833855, 1.8590057724288205, 1.864046048397789, 1.8690999899412386,
    1.8741676341103, 1.8792490180565602, 1.8843441790323345, 1.8894531543909392,
    1.8945759815869656, 1.8997126981765553, 1.9048633418176741, 1.9100279502703899,
    1.9152065613971474, 1.9203992131630474, 1.925605943636125, 1.930826790987627,
    1.9360617934922943, 1.9413109895286405, 1.9465744175792332, 1.9518521162309783,
    1.9571441241754002, 1.9624504802089273, 1.9677712232331759, 1.9731063922552343,
    1.978456026387951, 1.9838201648502194, 1.9891988469672663, 1.9945921121709402,
};
// a_k = (ln2/256)^k / k!, k = 1..4
static constexpr double kExpTabA256[4] = {0.0027076061740622863, 3.6655655969101062e-06, 3.3083026805413713e-09, 2.239395190875157e-12};
static constexpr double kInvLn2x256 = 369.3299304675746;   // 256 / ln2

// IS3D_EXP_TAB_BITS = 8 (default): 256-entry table, |c rs| <= ln2/512, degree-4 Taylor (truncation
// 3.8e-17): one FMA fewer per exp than the 64-entry table's degree 5; 6: the 64-entry table
#ifndef IS3D_EXP_TAB_BITS
#define IS3D_EXP_TAB_BITS 8
#endif
#if IS3D_EXP_TAB_BITS == 8
static constexpr int kExpTabN = 256, kExpTabDeg = 4;
#define kExp2Tab kExp2Tab256
#define kExpTabCoefs kExpTabA256
static constexpr double kInvLn2xN = kInvLn2x256;
#else
static constexpr int kExpTabN = 64, kExpTabDeg = 5;
#define kExp2Tab kExp2Tab64
#define kExpTabCoefs kExpTabA
static constexpr double kInvLn2xN = kInvLn2x64;
#endif

// degree of the modified lanes' 2^(r/N) polynomial with the 256-entry table: 3 (minimax, 3.5e-14 relative) or 4 (Taylor, ~1 ulp)
#ifndef IS3D_MOD_EXP_DEG
#define IS3D_MOD_EXP_DEG 3
#endif
// the modified lanes' exp table: IS3D_MOD_TAB_BITS = 8 shares exp_tab's 256 entries (degree-3 polynomial); 11 gives them
// their own 2^(j/2048) table (16 KB of LDS in the modified launches, which in turn drop their unused {b', Phi} rows:
// IS3D_MOD_TABLES) and a degree-2 polynomial -- one FMA fewer per point, 2.1e-13 instead of 3.5e-14 relative
#ifndef IS3D_MOD_TAB_BITS
#define IS3D_MOD_TAB_BITS 8
#endif
// the modified launch builds only the per-tile tables its lanes read: no {b', Phi} rows and no separable y-term
// slots (those serve the F_FB launch, which builds its own)
#ifndef IS3D_MOD_TABLES
#define IS3D_MOD_TABLES 1
#endif
#if IS3D_MOD_TAB_BITS == 11
#if !IS3D_MOD_TABLES
#error "IS3D_MOD_TAB_BITS = 11 needs IS3D_MOD_TABLES (the modified launches then read no exp_tab table)"
#endif
#include "exp2_tab2048.h"
static constexpr int kModTabN = 2048, kModExpDeg = 2;
#define kModExp2Tab kExp2Tab2048
static constexpr double kModInvLn2xN = kInvLn2x2048;
#define kModExpA kExpTabA2048
#elif IS3D_MOD_TAB_BITS == IS3D_EXP_TAB_BITS
static constexpr int kModTabN = kExpTabN;
#define kModExp2Tab kExp2Tab
static constexpr double kModInvLn2xN = kInvLn2xN;
#if IS3D_EXP_TAB_BITS == 8 && IS3D_MOD_EXP_DEG == 3
static constexpr int kModExpDeg = 3;
// near-minimax (Chebyshev) coefficients of (2^(r/256) - 1) / r on |r| <= 1/2: 1 + r p(r) within 3.5e-14
static constexpr double kModExpA[3] = {0.0027076061740622863, 3.6655660167967235e-06, 3.308302907918888e-09};
#else
static constexpr int kModExpDeg = kExpTabDeg;
#define kModExpA kExpTabCoefs
#endif
#else
#error "IS3D_MOD_TAB_BITS: 11, or equal to IS3D_EXP_TAB_BITS"
#endif

struct ExpTabCoef { double shift, a[kExpTabDeg]; };

IS3D_HD ExpTabCoef exp_tab_coef() {
  ExpTabCoef e;
  e.shift = kconst(6755399441055744.0);                  // 1.5 * 2^52
  for (int i = 0; i < kExpTabDeg; i++) e.a[i] = kconst(kExpTabCoefs[i]);
  return e;
}

// e^x 2^-kshift (exact shift, no intermediate overflow); xN = x kExpTabN/ln2
IS3D_HD double exp_tab(const ExpTabCoef& E, const double* tab, double xN, int kshift = 0) {
  const double t = xN + E.shift;
  const double K = t - E.shift;
  const double rs = xN - K;
  const int ki = (int)(unsigned)__builtin_bit_cast(unsigned long long, t);
  double q = E.a[kExpTabDeg - 1];
#pragma unroll
  for (int i = kExpTabDeg - 2; i >= 0; i--) q = fma(q, rs, E.a[i]);
  const double T = tab[ki & (kExpTabN - 1)];
  return ldexp(fma(T, rs * q, T), (ki >> IS3D_EXP_TAB_BITS) - kshift);
}

// e^(a v ln2 / kExpTabN) for a product a v (|a v| < 2^51) with the range reduction folded into the
// product: t = fma(a, v, shift) rounds a v to the integer K exactly (one rounding), shift - t = -K
// exactly, and rs = fma(a, v, -K) is the remainder with a single rounding -- three ops where
// xN = a v, xN + shift, t - shift, xN - K took four (modified path, mod_en_x)
IS3D_HD double exp_tab_fma(const ExpTabCoef& E, const double* tab, double a, double v) {
  const double t = fma(a, v, E.shift);
  const double rs = fma(a, v, E.shift - t);
  const int ki = (int)(unsigned)__builtin_bit_cast(unsigned long long, t);
  double q = E.a[kExpTabDeg - 1];
#pragma unroll
  for (int i = kExpTabDeg - 2; i >= 0; i--) q = fma(q, rs, E.a[i]);
  const double T = tab[ki & (kExpTabN - 1)];
  return ldexp(fma(T, rs * q, T), ki >> IS3D_EXP_TAB_BITS);
}

// sinh and cosh of d for the y-terms: |d| < 0.5 by their Taylor series through d^17 / d^16 (truncation
// < 5e-20 relative), otherwise from e = e^d and 1/e (e -/+ 1/e loses at most a factor coth(0.5) = 2.2 in
// relative accuracy): ~25 VALU ops instead of the library's double-double sinh / cosh (~100 each)
IS3D_HD void sinh_cosh(double d, double* sh, double* ch) {
  if (fabs(d) < 0.5) {
    const double d2 = d * d;
    double ps = kconst(1.0 / 355687428096000.0), pc = kconst(1.0 / 20922789888000.0);   // 1/17!, 1/16!
    const double fs[8] = {1.0 / 1307674368000.0, 1.0 / 6227020800.0, 1.0 / 39916800.0, 1.0 / 362880.0,
                          1.0 / 5040.0, 1.0 / 120.0, 1.0 / 6.0, 1.0};
    const double fc[8] = {1.0 / 87178291200.0, 1.0 / 479001600.0, 1.0 / 3628800.0, 1.0 / 40320.0,
                          1.0 / 720.0, 1.0 / 24.0, 0.5, 1.0};
    // coefficients pinned to SGPRs at the point of use (kconst): hoisted into VGPRs they were spilled
    for (int i = 0; i < 8; i++) { ps = fma(ps, d2, kconst(fs[i])); pc = fma(pc, d2, kconst(fc[i])); }
    *sh = d * ps;
    *ch = pc;
    return;
  }
  const double e = exp_dom690(d);
  const double r = 1.0 / e;
  *sh = 0.5 * (e - r);
  *ch = 0.5 * (e + r);
}

// exp(x) for any x: clamped into [-746, 710] first; ldexp saturates to +inf above 709.78 (the
// reference's exp overflow, after which 1/(inf + sign) = 0) and rounds to subnormal / zero below
// -708.4
IS3D_HD double exp_clamped(const ExpCoef& E, double x) { return exp_poly(E, fmin(fmax(x, -746.0), 710.0)); }

// 16-byte pair for ds_read_b128 of the phi-term rows (96-byte, 16-byte aligned)
#if defined(__HIP_DEVICE_COMPILE__)
typedef double dbl2 __attribute__((ext_vector_type(2)));
#else
struct alignas(16) dbl2 { double x, y; };
#endif

enum DfMode : int { GRAD = 1, CE = 2, PTM = 3, PTB = 4, PTMA = 5 };

static constexpr double kHbarC = 0.197327053;            // iS3D.h:14

// ---------------------------------------------------------------------------
// Per-cell record (output of the prepass, input of the spectra kernel), stored as an array of
// records rec[cell][NREC] so a tile of consecutive cells is one contiguous block.
// ---------------------------------------------------------------------------
enum Rec : int {
  R_KIND = 0,   // 0 skip (u.dsigma<=0), 1 separable (Grad/CE or breakdown), 2 modified
  R_T, R_INVT, R_CHEM,  // T (GeV), 1/T and alphaB entering feq (chem = baryon * R_CHEM)
  R_INVTM, R_CHEMM,  // 1/T_mod (1/lambda for PTMA) and alphaB_mod (upsilonB)
  R_TAU, R_ETA,
  R_UT, R_TAUUN, R_UX, R_UY,
  R_DAT, R_DANT, R_DAX, R_DAY,
  R_PITT, R_T2PINN, R_TPITN, R_PITX, R_PITY, R_TPIXN, R_TPIYN, R_PIXX, R_PIXY, R_PIYY,
  R_VT, R_TVN, R_VX, R_VY,
  R_SHEAR, R_BULK0, R_BULK1, R_BULK2, R_DIFF0, R_DIFF1, R_DLAM, R_DZ,
  R_ETASCALE, R_DET, R_NARROW, R_RENORM, R_ZB, R_VB,
  R_UCX, R_UCY, R_UCZ, R_USX, R_USY, R_USZ, R_VCX, R_VCY, R_VCZ, R_VSX, R_VSY, R_VSZ,
  // species-independent pieces of the separable lane coefficients (sep_cell_consts)
  R_S0M2, R_SCB, R_SSB, R_L0B, R_LC, R_LS,
  NREC
};
static_assert(NREC % 2 == 0, "records are moved as 16-byte pairs: keep NREC even");

// y-term layout (per cell, q); phi-terms are dbl2 pairs, see phiterms
// Y_AT = A/T, Y_A = A (u.p = mT A - pT B), Y_D (p.dsigma = mT D + ...), Y_WDX/Y_WDY = w_eta dsigma_{x,y};
// Y_S2, Y_S1, Y_SC1, Y_SS1, Y_L1: the (cell, y) factors of the separable lane coefficients
// (sep_setup); Y_MUX..Y_MD, Y_NARROW, Y_MU2 = |sig U|^2, Y_MU = |sig U|: modified-momentum path.
enum YT : int { Y_AT = 0, Y_A, Y_D, Y_WDX, Y_WDY, Y_S2, Y_S1, Y_SC1, Y_SS1, Y_L1,
                Y_MUX, Y_MUY, Y_MUZ, Y_MD, Y_NARROW, Y_W, Y_MU2, Y_MU, NYT };

// surface field order (include/is3d_amd.h, is3d_surface)
enum Surf : int {
  S_TAU = 0, S_X, S_Y, S_ETA, S_DAT, S_DAX, S_DAY, S_DAN, S_UX, S_UY, S_UN, S_E, S_T, S_P,
  S_PIXX, S_PIXY, S_PIXN, S_PIYY, S_PIYN, S_BULKPI, S_MUB, S_NB, S_VX, S_VY, S_VN, NSURF
};

// ---------------------------------------------------------------------------
// delta-f coefficient tables (DeltafData.cpp)
// ---------------------------------------------------------------------------
enum Spl : int { SP_C0 = 0, SP_C2, SP_C3, SP_F, SP_BB, SP_BV, SP_BP, NSPL };

struct DfTables {
  int df_mode, include_baryon;
  int nT, nmuB;
  const double *T, *muB, *tab;           // tab[10][nmuB][nT]
  double T_min, muB_min, dT, dmuB;
  const double *sy[NSPL], *sc[NSPL];     // spline knot values / second-derivative coefficients (x = T)
  int nj;                                // Jonah table (PTB)
  const double *jx, *jl2, *jl2c, *jz, *jzc;
  double bulk_over_P_max;
};

struct DfCoef {
  double c0, c1, c2, c3, c4, shear14, F, G, betabulk, betaV, betapi, lambda, z, dlambda, dz;
};

enum DfErr : int { DF_OK = 0, DF_SPLINE_RANGE = 1, DF_BAD_MODE = 2, DF_TABLE_RANGE = 3, DF_PTB_BARYON = 4, DF_TS_SLOW = 5 };

// gsl_spline_eval for gsl_interp_cspline: range check, binary search, coeff_calc
IS3D_HD double spline_eval(const double* x, const double* y, const double* c, int n, double xv, int* err) {
  if (xv < x[0] || xv > x[n - 1]) { *err = DF_SPLINE_RANGE; return 0.0; }
  int lo = 0, hi = n - 1;
  while (hi > lo + 1) { int i = (hi + lo) >> 1; if (x[i] > xv) hi = i; else lo = i; }
  const double dx = x[lo + 1] - x[lo];
  if (!(dx > 0.0)) return 0.0;
  const double dy = y[lo + 1] - y[lo], delx = xv - x[lo];
  const double ci = c[lo], cip1 = c[lo + 1];
  const double b = (dy / dx) - dx * (cip1 + 2.0 * ci) / 3.0;
  const double d = (cip1 - ci) / (3.0 * dx);
  return y[lo] + delx * (b + delx * (ci + delx * d));
}

IS3D_HD double tabv(const DfTables& t, int k, int iB, int iT) { return t.tab[((long)k * t.nmuB + iB) * t.nT + iT]; }

IS3D_HD double bilinear(const DfTables& t, int k, double T, double muB, double TL, double TR, double mL, double mR,
                        int iTL, int iTR, int imL, int imR) {
  const double fLL = tabv(t, k, imL, iTL), fLR = tabv(t, k, imR, iTL), fRL = tabv(t, k, imL, iTR), fRR = tabv(t, k, imR, iTR);
  return ((fLL * (TR - T) + fRL * (T - TL)) * (mR - muB) + (fLR * (TR - T) + fRR * (T - TL)) * (muB - mL)) / (t.dT * t.dmuB);
}

// Deltaf_Data::evaluate_df_coefficients (DeltafData.cpp:324-519)
IS3D_HD int df_eval(const DfTables& t, double T, double muB, double E, double P, double bulkPi, DfCoef& df) {
  df = DfCoef{0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0};
  int err = DF_OK;
  const double T4 = T * T * T * T;
  if (!t.include_baryon) {
    switch (t.df_mode) {
      case GRAD:
        df.c0 = spline_eval(t.T, t.sy[SP_C0], t.sc[SP_C0], t.nT, T, &err) / T4;
        df.c2 = spline_eval(t.T, t.sy[SP_C2], t.sc[SP_C2], t.nT, T, &err) / T4;
        df.shear14 = 2.0 * T * T * (E + P);
        break;
      case CE: case PTM: case PTMA:
        df.F = spline_eval(t.T, t.sy[SP_F], t.sc[SP_F], t.nT, T, &err) * T;
        df.betabulk = spline_eval(t.T, t.sy[SP_BB], t.sc[SP_BB], t.nT, T, &err) * T4;
        df.betaV = 1.0;
        df.betapi = spline_eval(t.T, t.sy[SP_BP], t.sc[SP_BP], t.nT, T, &err) * T4;
        break;
      case PTB: {
        const double l2 = spline_eval(t.jx, t.jl2, t.jl2c, t.nj, bulkPi / P, &err);
        df.lambda = 0.0;  // reference leaves lambda uninitialised when bulkPi == 0
        if (bulkPi < 0.0) df.lambda = -sqrt(l2);
        else if (bulkPi > 0.0) df.lambda = sqrt(l2);
        df.z = spline_eval(t.jx, t.jz, t.jzc, t.nj, bulkPi / P, &err);
        df.betapi = spline_eval(t.T, t.sy[SP_BP], t.sc[SP_BP], t.nT, T, &err) * T4;
        df.dlambda = bulkPi / (5.0 * df.betapi - 3.0 * P * (E + P) / E);
        df.dz = -3.0 * df.dlambda * P / E;
        break;
      }
      default: return DF_BAD_MODE;
    }
    return err;
  }
  const int iTL = (int)floor((T - t.T_min) / t.dT), iTR = iTL + 1;
  const int imL = (int)floor((muB - t.muB_min) / t.dmuB), imR = imL + 1;
  if (!(iTL >= 0 && iTR < t.nT) || !(imL >= 0 && imR < t.nmuB)) return DF_TABLE_RANGE;
  const double TL = t.T[iTL], TR = t.T[iTR], mL = t.muB[imL], mR = t.muB[imR];
  const double T3 = T * T * T, T5 = T4 * T;
  switch (t.df_mode) {
    case GRAD:
      df.c0 = bilinear(t, 0, T, muB, TL, TR, mL, mR, iTL, iTR, imL, imR) / T4;
      df.c1 = bilinear(t, 1, T, muB, TL, TR, mL, mR, iTL, iTR, imL, imR) / T3;
      df.c2 = bilinear(t, 2, T, muB, TL, TR, mL, mR, iTL, iTR, imL, imR) / T4;
      df.c3 = bilinear(t, 3, T, muB, TL, TR, mL, mR, iTL, iTR, imL, imR) / T4;
      df.c4 = bilinear(t, 4, T, muB, TL, TR, mL, mR, iTL, iTR, imL, imR) / T5;
      df.shear14 = 2.0 * T * T * (E + P);
      break;
    case CE: case PTM: case PTMA:
      df.F = bilinear(t, 5, T, muB, TL, TR, mL, mR, iTL, iTR, imL, imR) * T;
      df.G = bilinear(t, 6, T, muB, TL, TR, mL, mR, iTL, iTR, imL, imR);
      df.betabulk = bilinear(t, 7, T, muB, TL, TR, mL, mR, iTL, iTR, imL, imR) * T4;
      df.betaV = bilinear(t, 8, T, muB, TL, TR, mL, mR, iTL, iTR, imL, imR) * T3;
      df.betapi = bilinear(t, 9, T, muB, TL, TR, mL, mR, iTL, iTR, imL, imR) * T4;
      break;
    case PTB: return DF_PTB_BARYON;
    default: return DF_BAD_MODE;
  }
  return DF_OK;
}

// ---------------------------------------------------------------------------
// PTB "Jonah" table (DeltafData.cpp:220-295 compute_jonah_coefficients): 301 lambda rows in
// [-1, 2]; per row the HRG kinetic E, P at lambda = 0 and at lambda over the PDG (photon skipped).
// Built on the device (k_jonah_terms / k_jonah_sum) and by the test emulator from these pieces;
// no FMA contraction here, so the device table is bit-identical to the host's (and the reference
// expression order is kept: lmin + i dl rounds the product first).
// ---------------------------------------------------------------------------
static constexpr int kJonahN = 301;

IS3D_HD double jonah_lambda(int i) {
#pragma clang fp contract(off)
  const double lmin = -1.0, lmax = 2.0, dl = (lmax - lmin) / ((double)kJonahN - 1.0);
  return lmin + (double)i * dl;
}

// E_mod_int (kind 0) / P_mod_int (kind 1) Gauss sums (GaussThermal.cpp:108-130)
IS3D_HD double gauss1d_mod(int kind, const double* r, const double* w, int n, double mbar, double lambda, double sign) {
#pragma clang fp contract(off)
  const ExpCoef E = exp_coef();
  double sum = 0.0;
  for (int k = 0; k < n; k++) {
    const double p = r[k], scale2 = (1.0 + lambda) * (1.0 + lambda), Eb = sqrt(p * p + mbar * mbar);
    const double v = (kind == 0) ? sqrt(p * p * scale2 + mbar * mbar) * exp_clamped(E, p) / (exp_clamped(E, Eb) + sign)
                                 : p * p * scale2 / sqrt(p * p * scale2 + mbar * mbar) * exp_clamped(E, p) / (exp_clamped(E, Eb) + sign);
    sum += w[k] * v;
  }
  return sum;
}

// one hadron's terms of a row: g E_mod and g P_mod / 3 (0 for m = 0: the reference skips the photon)
IS3D_HD void jonah_terms(double T, double mass, double degen, double sign, const double* r2, const double* w2, int pts,
                         double lambda, double* em, double* pm) {
#pragma clang fp contract(off)
  if (mass == 0.0) { *em = 0.0; *pm = 0.0; return; }
  const double mbar = mass / T;
  *em = degen * gauss1d_mod(0, r2, w2, pts, mbar, lambda, sign);
  *pm = (1.0 / 3.0) * degen * gauss1d_mod(1, r2, w2, pts, mbar, lambda, sign);
}

// row i from the hadron sums (E, P at lambda = 0; Em, Pm at lambda): lambda^2, z, bulkPi/P
IS3D_HD void jonah_row(int i, double E, double P, double Em, double Pm, double* l2, double* z, double* bp) {
#pragma clang fp contract(off)
  const double lambda = jonah_lambda(i);
  const double zz = E / Em;
  l2[i] = lambda * lambda;
  z[i] = zz;
  bp[i] = (Pm / P) * zz - 1.0;
}

// ---------------------------------------------------------------------------
// Gauss-Laguerre thermal integrals (GaussThermal.cpp:7-78)
// ---------------------------------------------------------------------------
IS3D_HD double gt_neq(const double* r, const double* w, int n, double mbar, double alphaB, double baryon, double sign) {
  double s = 0.0;
  for (int k = 0; k < n; k++) {
    const double p = r[k], Eb = sqrt(p * p + mbar * mbar);
    s += w[k] * (p * exp(p) / (exp(Eb - baryon * alphaB) + sign));
  }
  return s;
}
IS3D_HD double gt_J10(const double* r, const double* w, int n, double mbar, double alphaB, double baryon, double sign) {
  double s = 0.0;
  for (int k = 0; k < n; k++) {
    const double p = r[k], Eb = sqrt(p * p + mbar * mbar), q = exp(Eb - baryon * alphaB) + sign;
    s += w[k] * (p * exp(p + Eb - baryon * alphaB) / (q * q));
  }
  return s;
}
IS3D_HD double gt_J20(const double* r, const double* w, int n, double mbar, double alphaB, double baryon, double sign) {
  double s = 0.0;
  for (int k = 0; k < n; k++) {
    const double p = r[k], Eb = sqrt(p * p + mbar * mbar), q = exp(Eb - baryon * alphaB) + sign;
    s += w[k] * (Eb * exp(p + Eb - baryon * alphaB) / (q * q));
  }
  return s;
}

// ---------------------------------------------------------------------------
// 3x3 helpers: LU with partial pivoting (gsl_linalg_LU_decomp/_solve/_invert)
// ---------------------------------------------------------------------------
IS3D_HD void lu3_decomp(double* A, int* perm) {
  perm[0] = 0; perm[1] = 1; perm[2] = 2;
  for (int j = 0; j < 3; j++) {
    int piv = j; double mx = fabs(A[3 * j + j]);
    for (int i = j + 1; i < 3; i++) if (fabs(A[3 * i + j]) > mx) { mx = fabs(A[3 * i + j]); piv = i; }
    if (piv != j) {
      for (int k = 0; k < 3; k++) { const double t = A[3 * j + k]; A[3 * j + k] = A[3 * piv + k]; A[3 * piv + k] = t; }
      const int t = perm[j]; perm[j] = perm[piv]; perm[piv] = t;
    }
    const double ajj = A[3 * j + j];
    if (ajj != 0.0) {
      for (int i = j + 1; i < 3; i++) {
        const double aij = A[3 * i + j] / ajj;
        A[3 * i + j] = aij;
        for (int k = j + 1; k < 3; k++) A[3 * i + k] -= aij * A[3 * j + k];
      }
    }
  }
}

IS3D_HD void lu3_solve(const double* LU, const int* perm, const double* b, double* x) {
  double y[3];
  for (int i = 0; i < 3; i++) y[i] = b[perm[i]];
  for (int i = 0; i < 3; i++) { double s = y[i]; for (int k = 0; k < i; k++) s -= LU[3 * i + k] * y[k]; y[i] = s; }
  for (int i = 2; i >= 0; i--) { double s = y[i]; for (int k = i + 1; k < 3; k++) s -= LU[3 * i + k] * x[k]; x[i] = s / LU[3 * i + i]; }
}

// A^{-1} applied to the four LRF basis directions -> Uc, Us, Vc, Vs (written to rec R_UCX..R_VSZ)
IS3D_HD void modified_directions(const double* Asym, double tau, double Xt, double Xx, double Xy, double Xn,
                                 double Yx, double Yy, double Zt, double Zn, double* rec_u /* 12 */) {
  double LU[9]; int perm[3];
  for (int i = 0; i < 9; i++) LU[i] = Asym[i];
  lu3_decomp(LU, perm);
  const double dirs[4][3] = {{-Xt, 0.0, -Zt}, {tau * Xn, 0.0, tau * Zn}, {Xx, Yx, 0.0}, {Xy, Yy, 0.0}};
  for (int d = 0; d < 4; d++) lu3_solve(LU, perm, dirs[d], rec_u + 3 * d);
}

// Last step of the modified-path prologues (R_INVTM, R_CHEMM, R_VB and the directions set): Uc, Us, Vc,
// Vs and R_VB in the modified lanes' exp-table units, scaled by sig = (1/T_mod) kModTabN/ln2, so that every
// E_mod^2 the lanes build (mod_setup, modqv, modt2) is (sig E_mod)^2 and its square root is their exp's argument
// without a multiply
IS3D_HD void mod_scale_record(double* R) {
  const double sig = R[R_INVTM] * kModInvLn2xN;
  for (int f = R_UCX; f <= R_VSZ; f++) R[f] *= sig;
  R[R_VB] *= sig;
}

// ---------------------------------------------------------------------------
// Milne basis / LRF boosts (LocalRestFrame.cpp:12-41, 133-154)
// ---------------------------------------------------------------------------
struct Milne { double Xt, Xx, Xy, Xn, Yx, Yy, Zt, Zn; };

IS3D_HD Milne milne_basis(double ut, double ux, double uy, double un, double uperp, double utperp, double tau) {
  Milne b;
  const double sinhL = tau * un / utperp, coshL = ut / utperp;
  b.Xt = uperp * coshL; b.Xx = 1; b.Xy = 0; b.Xn = uperp * sinhL / tau;
  b.Yx = 0; b.Yy = 1; b.Zt = sinhL; b.Zn = coshL / tau;
  if (uperp > 1.e-5) {
    b.Xx = utperp * ux / uperp; b.Xy = utperp * uy / uperp;
    b.Yx = -uy / uperp; b.Yy = ux / uperp;
  }
  return b;
}

struct PiLRF { double xx, xy, xz, yy, yz, zz; };

IS3D_HD PiLRF boost_pi(const Milne& b, double tau2, double pitt, double pitx, double pity, double pitn, double pixx,
                       double pixy, double pixn, double piyy, double piyn, double pinn) {
  PiLRF r;
  const double Xt = b.Xt, Xx = b.Xx, Xy = b.Xy, Xn = b.Xn, Yx = b.Yx, Yy = b.Yy, Zt = b.Zt, Zn = b.Zn;
  r.xx = pitt * Xt * Xt + pixx * Xx * Xx + piyy * Xy * Xy + tau2 * tau2 * pinn * Xn * Xn +
         2.0 * (-Xt * (pitx * Xx + pity * Xy) + pixy * Xx * Xy + tau2 * Xn * (pixn * Xx + piyn * Xy - pitn * Xt));
  r.xy = Yx * (-pitx * Xt + pixx * Xx + pixy * Xy + tau2 * pixn * Xn) + Yy * (-pity * Xt + pixy * Xx + piyy * Xy + tau2 * piyn * Xn);
  r.xz = Zt * (pitt * Xt - pitx * Xx - pity * Xy - tau2 * pitn * Xn) - tau2 * Zn * (pitn * Xt - pixn * Xx - piyn * Xy - tau2 * pinn * Xn);
  r.yy = pixx * Yx * Yx + 2.0 * pixy * Yx * Yy + piyy * Yy * Yy;
  r.yz = -Zt * (pitx * Yx + pity * Yy) + tau2 * Zn * (pixn * Yx + piyn * Yy);
  r.zz = -(r.xx + r.yy);
  return r;
}

// ---------------------------------------------------------------------------
// Run-level constants for the prepass
// ---------------------------------------------------------------------------
struct PrepConsts {
  int operation;   // 1 continuous spectra, 0 spacetime distributions (differences: see yterms / prep_*)
  int df_mode, dim, include_baryon, include_bulk, include_shear, include_diff;
  double deta_min, mass_pion0;
  int gla_pts;
  const double *gla_r1, *gla_w1, *gla_r2, *gla_w2;
  double two_pi2_hbarC3;
  double pT_max, b_max;   // momentum grid's largest pT, species' largest |baryon| (sep_slow_cell)
};

// common fields for every record
IS3D_HD void rec_common(double* R, double tau, double eta, double ut, double un, double ux, double uy, double dat,
                        double dax, double day, double dan, double T) {
  R[R_TAU] = tau; R[R_ETA] = eta; R[R_UT] = ut; R[R_TAUUN] = tau * un; R[R_UX] = ux; R[R_UY] = uy;
  R[R_DAT] = dat; R[R_DANT] = dan / tau; R[R_DAX] = dax; R[R_DAY] = day; R[R_T] = T; R[R_INVT] = 1.0 / T;
  R[R_ZB] = sqrt(ux * ux + uy * uy) / T;
}

IS3D_HD void rec_pi(double* R, double tau, double pitt, double pitx, double pity, double pitn, double pixx, double pixy,
                    double pixn, double piyy, double piyn, double pinn) {
  R[R_PITT] = pitt; R[R_T2PINN] = tau * tau * pinn; R[R_TPITN] = tau * pitn; R[R_PITX] = pitx; R[R_PITY] = pity;
  R[R_TPIXN] = tau * pixn; R[R_TPIYN] = tau * piyn; R[R_PIXX] = pixx; R[R_PIXY] = pixy; R[R_PIYY] = piyy;
}

// --- Grad / RTA-CE prologue (MomentumSpectra.cpp:109-246) ---
IS3D_HD int prep_grad_ce(const PrepConsts& k, const DfTables& tb, const double* s, double* R) {
  for (int f = 0; f < NREC; f++) R[f] = 0.0;
  const double tau = s[S_TAU], tau2 = tau * tau;
  const double eta = (k.dim == 3) ? s[S_ETA] : 0.0;
  const double dat = s[S_DAT], dax = s[S_DAX], day = s[S_DAY], dan = s[S_DAN];
  const double ux = s[S_UX], uy = s[S_UY], un = s[S_UN];
  const double ux2 = ux * ux, uy2 = uy * uy, utperp = sqrt(1.0 + ux2 + uy2), tau2_un = tau2 * un;
  const double ut = sqrt(utperp * utperp + tau2_un * un), ut2 = ut * ut;
  if (ut * dat + ux * dax + uy * day + un * dan <= 0.0) { R[R_KIND] = 0.0; return DF_OK; }
  const double T = s[S_T], P = s[S_P], E = s[S_E];
  double pitt = 0, pitx = 0, pity = 0, pitn = 0, pixx = 0, pixy = 0, pixn = 0, piyy = 0, piyn = 0, pinn = 0;
  if (k.include_shear) {
    pixx = s[S_PIXX]; pixy = s[S_PIXY]; pixn = s[S_PIXN]; piyy = s[S_PIYY]; piyn = s[S_PIYN];
    pinn = (pixx * (ux2 - ut2) + piyy * (uy2 - ut2) + 2.0 * (pixy * ux * uy + tau2_un * (pixn * ux + piyn * uy))) / (tau2 * utperp * utperp);
    pitn = (pixn * ux + piyn * uy + tau2_un * pinn) / ut;
    pity = (pixy * ux + piyy * uy + tau2_un * piyn) / ut;
    pitx = (pixx * ux + pixy * uy + tau2_un * pixn) / ut;
    pitt = (pitx * ux + pity * uy + tau2_un * pitn) / ut;
  }
  const double bulkPi = k.include_bulk ? s[S_BULKPI] : 0.0;
  double muB = 0, alphaB = 0, nB = 0, Vt = 0, Vx = 0, Vy = 0, Vn = 0, ber = 0;
  if (k.include_baryon && k.include_diff) {
    muB = s[S_MUB]; nB = s[S_NB]; Vx = s[S_VX]; Vy = s[S_VY]; Vn = s[S_VN];
    Vt = (Vx * ux + Vy * uy + Vn * tau2_un) / ut;
    alphaB = muB / T;
    ber = nB / (E + P);
  }
  DfCoef df;
  const int err = df_eval(tb, T, muB, E, P, bulkPi, df);
  if (err) return err;
  rec_common(R, tau, eta, ut, un, ux, uy, dat, dax, day, dan, T);
  rec_pi(R, tau, pitt, pitx, pity, pitn, pixx, pixy, pixn, piyy, piyn, pinn);
  // V^mu is nonzero only with include_baryon && include_diff; with include_baryon = 0 it and c1 = c3 = 0
  // (df_eval) make sep_cell_consts' R_SCB = R_SSB = 0, which the F_TB launch relies on (engine.hip)
  R[R_VT] = Vt; R[R_TVN] = tau * Vn; R[R_VX] = Vx; R[R_VY] = Vy;
  R[R_CHEM] = alphaB;
  if (k.df_mode == GRAD) {
    // 1 / (2 T^2 (E+P)) written as in each path (MomentumSpectra.cpp:215, SpacetimeDistribution.cpp:269)
    R[R_SHEAR] = (k.operation == 0) ? 0.5 / (T * T * (E + P)) : 1.0 / df.shear14;
    R[R_BULK0] = (df.c0 - df.c2) * bulkPi; R[R_BULK1] = df.c1 * bulkPi; R[R_BULK2] = (4. * df.c2 - df.c0) * bulkPi;
    R[R_DIFF0] = df.c3; R[R_DIFF1] = df.c4;
  } else {
    R[R_SHEAR] = 0.5 / (df.betapi * T);
    R[R_BULK0] = df.F / (T * T * df.betabulk) * bulkPi; R[R_BULK1] = df.G / df.betabulk * bulkPi;
    R[R_BULK2] = bulkPi / (3.0 * T * df.betabulk);
    R[R_DIFF0] = ber / df.betaV; R[R_DIFF1] = 1.0 / df.betaV;
  }
  R[R_ETASCALE] = 1.0;
  R[R_KIND] = 1.0;
  return DF_OK;
}

// --- PTM / PTB prologue (MomentumSpectra.cpp:516-773 + EmissionFunction.cpp:65-109) ---
// stats[0] += breakdown, stats[1] += pl<0.  renorm_base: PTM -> 1/den (species factor from the
// renorm kernel), PTB -> z/den.  aux[0..3] = T, T_mod, alphaB, alphaB_mod and aux[4..6] = F, G,
// betabulk and aux[7] bulkPi (for the PTM renorm kernel).
IS3D_HD int prep_feqmod(const PrepConsts& k, const DfTables& tb, const double* s, double* R, double* aux, int* flags) {
  for (int f = 0; f < NREC; f++) R[f] = 0.0;
  flags[0] = flags[1] = 0;
  const double tau = s[S_TAU], tau2 = tau * tau;
  const double eta = (k.dim == 3) ? s[S_ETA] : 0.0;
  const double dat = s[S_DAT], dax = s[S_DAX], day = s[S_DAY], dan = s[S_DAN];
  const double ux = s[S_UX], uy = s[S_UY], un = s[S_UN];
  const double ut = sqrt(1.0 + ux * ux + uy * uy + tau2 * un * un);
  if (ut * dat + ux * dax + uy * day + un * dan <= 0.0) { R[R_KIND] = 0.0; return DF_OK; }
  const double ut2 = ut * ut, ux2 = ux * ux, uy2 = uy * uy;
  const double uperp = sqrt(ux * ux + uy * uy), utperp = sqrt(1.0 + ux * ux + uy * uy);
  const double T = s[S_T], P = s[S_P], E = s[S_E];
  double pitt = 0, pitx = 0, pity = 0, pitn = 0, pixx = 0, pixy = 0, pixn = 0, piyy = 0, piyn = 0, pinn = 0;
  if (k.include_shear) {
    pixx = s[S_PIXX]; pixy = s[S_PIXY]; pixn = s[S_PIXN]; piyy = s[S_PIYY]; piyn = s[S_PIYN];
    pinn = (pixx * (ux2 - ut2) + piyy * (uy2 - ut2) + 2.0 * (pixy * ux * uy + tau2 * un * (pixn * ux + piyn * uy))) / (tau2 * utperp * utperp);
    pitn = (pixn * ux + piyn * uy + tau2 * pinn * un) / ut;
    pity = (pixy * ux + piyy * uy + tau2 * piyn * un) / ut;
    pitx = (pixx * ux + pixy * uy + tau2 * pixn * un) / ut;
    pitt = (pitx * ux + pity * uy + tau2 * pitn * un) / ut;
  }
  double bulkPi = k.include_bulk ? s[S_BULKPI] : 0.0;
  double muB = 0, alphaB = 0, nB = 0, Vt = 0, Vx = 0, Vy = 0, Vn = 0, ber = 0;
  if (k.include_baryon && k.include_diff) {
    muB = s[S_MUB]; nB = s[S_NB]; Vx = s[S_VX]; Vy = s[S_VY]; Vn = s[S_VN];
    Vt = (Vx * ux + Vy * uy + tau2 * Vn * un) / ut;
    alphaB = muB / T;
    ber = nB / (E + P);
  }
  if (k.df_mode == PTB) {   // MomentumSpectra.cpp:603-615 (< / >); SpacetimeDistribution.cpp:766-772 (<= / >=)
    const bool lo = (k.operation == 0) ? (bulkPi <= -P) : (bulkPi < -P);
    const bool hi = (k.operation == 0) ? (bulkPi / P >= tb.bulk_over_P_max) : (bulkPi / P > tb.bulk_over_P_max);
    if (lo) bulkPi = -(1.0 - 1.e-5) * P;
    else if (hi) bulkPi = P * (tb.bulk_over_P_max - 1.e-5);
  }
  const double zt = tau * un / utperp, zn = ut / (tau * utperp);
  const double pl = P + bulkPi + zt * zt * pitt + tau2 * tau2 * zn * zn * pinn + 2. * tau2 * zt * zn * pitn;
  if (pl < 0) flags[1] = 1;
  DfCoef df;
  const int err = df_eval(tb, T, muB, E, P, bulkPi, df);
  if (err) return err;
  const double F = df.F, G = df.G, betabulk = df.betabulk, betaV = df.betaV, betapi = df.betapi;
  const Milne b = milne_basis(ut, ux, uy, un, uperp, utperp, tau);
  const PiLRF pl_ = boost_pi(b, tau2, pitt, pitx, pity, pitn, pixx, pixy, pixn, piyy, piyn, pinn);
  double T_mod = T, alphaB_mod = alphaB;
  if (k.df_mode == PTM) { T_mod = T + bulkPi * F / betabulk; alphaB_mod = alphaB + bulkPi * G / betabulk; }
  const double shear_coeff = 0.5 / (betapi * T);
  const double shear_mod = 0.5 / betapi;
  double bulk_mod = bulkPi / (3.0 * betabulk);
  if (k.df_mode == PTB) bulk_mod = df.lambda;
  const double Axx = 1.0 + pl_.xx * shear_mod + bulk_mod, Axy = pl_.xy * shear_mod, Axz = pl_.xz * shear_mod;
  const double Ayy = 1.0 + pl_.yy * shear_mod + bulk_mod, Ayz = pl_.yz * shear_mod, Azz = 1.0 + pl_.zz * shear_mod + bulk_mod;
  const double detA = Axx * (Ayy * Azz - Ayz * Ayz) - Axy * (Axy * Azz - Ayz * Axz) + Axz * (Axy * Ayz - Ayy * Axz);
  const double detA_b23 = pow(1.0 + bulk_mod, 2);
  const double A[9] = {Axx, Axy, Axz, Axy, Ayy, Ayz, Axz, Ayz, Azz};
  // breakdown test (EmissionFunction.cpp:65-109, fast = 0)
  int breaks = 0;
  if (k.df_mode == PTM) {
    const double mbar = k.mass_pion0 / T;
    const double neq_fact = T * T * T / k.two_pi2_hbarC3, J20_fact = T * neq_fact;
    const double neq = neq_fact * gt_neq(k.gla_r1, k.gla_w1, k.gla_pts, mbar, 0., 0., -1.);
    const double J20 = J20_fact * gt_J20(k.gla_r2, k.gla_w2, k.gla_pts, mbar, 0., 0., -1.);
    const double dn = bulkPi * (neq + J20 * F / T / T) / betabulk;
    breaks = (detA <= k.deta_min || (neq + dn < 0.0));
  } else {
    breaks = (detA <= k.deta_min || df.z < 0.0);
  }
  flags[0] = breaks;
  double eta_scale = 1.0;
  if (detA > k.deta_min && k.dim == 2) eta_scale = detA / detA_b23;
  const double den = (k.dim == 2) ? detA_b23 : detA;
  double renorm_base = 1.0;
  if (k.include_bulk && k.df_mode == PTB) renorm_base = df.z;
  rec_common(R, tau, eta, ut, un, ux, uy, dat, dax, day, dan, T);
  rec_pi(R, tau, pitt, pitx, pity, pitn, pixx, pixy, pixn, piyy, piyn, pinn);
  R[R_VT] = Vt; R[R_TVN] = tau * Vn; R[R_VX] = Vx; R[R_VY] = Vy;
  R[R_CHEM] = (k.df_mode == PTB) ? 0.0 : alphaB;   // PTB breakdown feq has no chemical potential (:913)
  R[R_INVTM] = 1.0 / T_mod; R[R_CHEMM] = alphaB_mod;
  R[R_SHEAR] = shear_coeff;
  if (k.df_mode == PTM) {   // linearised CE fallback (:887-909): same shape as CE
    R[R_BULK0] = F / (T * T * betabulk) * bulkPi; R[R_BULK1] = G / betabulk * bulkPi;
    R[R_BULK2] = 1.0 / (3.0 * T * betabulk) * bulkPi;
    R[R_DIFF0] = ber / betaV; R[R_DIFF1] = 1.0 / betaV;
  } else {
    R[R_DLAM] = df.dlambda; R[R_DZ] = df.dz;
  }
  R[R_ETASCALE] = eta_scale; R[R_DET] = detA;
  R[R_NARROW] = (k.dim == 3 && detA < 0.01) ? 1.0 : 0.0;
  R[R_RENORM] = renorm_base / den;
  modified_directions(A, tau, b.Xt, b.Xx, b.Xy, b.Xn, b.Yx, b.Yy, b.Zt, b.Zn, R + R_UCX);
  R[R_VB] = sqrt(R[R_VCX] * R[R_VCX] + R[R_VCY] * R[R_VCY] + R[R_VCZ] * R[R_VCZ]) +
            sqrt(R[R_VSX] * R[R_VSX] + R[R_VSY] * R[R_VSY] + R[R_VSZ] * R[R_VSZ]);
  mod_scale_record(R);
  aux[0] = T; aux[1] = T_mod; aux[2] = alphaB; aux[3] = alphaB_mod; aux[4] = F; aux[5] = G; aux[6] = betabulk; aux[7] = bulkPi;
  aux[8] = den;
  R[R_KIND] = breaks ? 1.0 : 2.0;
  return DF_OK;
}

// ---------------------------------------------------------------------------
// operation = 2 oversampling estimate (ParticleSampler.cpp:447-636 calculate_total_yield)
// ---------------------------------------------------------------------------
// The six GaussThermal integrands (GaussThermal.cpp:19-78) that compute_particle_densities
// (DeltafData.cpp:555-690) needs, at Gauss-Laguerre root p of the matching alpha.
IS3D_HD double gt_term(int kind, double p, double mbar, double chem, double sign) {
  const double Eb = sqrt(p * p + mbar * mbar);
  if (kind == 0) return p * exp(p) / (exp(Eb - chem) + sign);                 // neq   (a = 1)
  const double q = exp(Eb - chem) + sign, x = exp(p + Eb - chem) / (q * q);
  switch (kind) {
    case 1: return p * x;                                                       // J10   (a = 1)
    case 2: return p * p * p / (Eb * Eb) * x;                                   // J11   (a = 1)
    case 3: return Eb * x;                                                      // J20   (a = 2)
    case 4: return Eb * Eb / p * x;                                             // J30   (a = 3)
    default: return p * x;                                                      // J31   (a = 3)
  }
}

// equilibrium / bulk / diffusion densities of one species from its six thermal integrals
// J[0..5] = (neq, J10, J11, J20, J30, J31) integrals (before the T^n g / 2 pi^2 hbarc^3 factors)
IS3D_HD void species_densities(int df_mode, const DfCoef& df, double T, double ber, double mass, double degeneracy,
                               double baryon, const double* J, double two_pi2_hbarC3, double* out3) {
  const double neq = degeneracy * pow(T, 3) / two_pi2_hbarC3 * J[0];
  double dn_bulk = 0.0, dn_diff = 0.0;
  if (df_mode == GRAD) {
    const double J10 = degeneracy * pow(T, 3) / two_pi2_hbarC3 * J[1];
    const double J20 = degeneracy * pow(T, 4) / two_pi2_hbarC3 * J[3];
    const double J30 = degeneracy * pow(T, 5) / two_pi2_hbarC3 * J[4];
    const double J31 = degeneracy * pow(T, 5) / two_pi2_hbarC3 / 3.0 * J[5];
    dn_bulk = ((df.c0 - df.c2) * mass * mass * J10 + df.c1 * baryon * J20 + (4.0 * df.c2 - df.c0) * J30);
    dn_diff = baryon * df.c3 * neq * T + df.c4 * J31;
  } else if (df_mode != PTB) {   // CE, PTM and PTMA (goto chapman_enskog, :666-669)
    const double J10 = degeneracy * pow(T, 3) / two_pi2_hbarC3 * J[1];
    const double J11 = degeneracy * pow(T, 3) / two_pi2_hbarC3 / 3.0 * J[2];
    const double J20 = degeneracy * pow(T, 4) / two_pi2_hbarC3 * J[3];
    dn_bulk = (neq + (baryon * J10 * df.G) + (J20 * df.F / pow(T, 2))) / df.betabulk;
    dn_diff = (neq * T * ber - baryon * J11) / df.betaV;
  }
  out3[0] = neq; out3[1] = dn_bulk; out3[2] = dn_diff;
}

// Sum over chosen species of estimate_mean_particle_number (ParticleSampler.cpp:75-119) for one
// cell; dsum = species sums of the (equilibrium, bulk, diffusion) densities, which the estimate is
// linear in.  Returns 0 for cells with u.dsigma <= 0.  ds_space per compute_dsigma_magnitude
// (the reference reads that member without calling it, :582-583: uninitialised).
IS3D_HD int yield_cell(const PrepConsts& k, const DfTables& tb, const double* s, const double* dsum, double* out) {
  *out = 0.0;
  const double tau = s[S_TAU], tau2 = tau * tau;
  const double dat = s[S_DAT], dax = s[S_DAX], day = s[S_DAY], dan = s[S_DAN];
  const double ux = s[S_UX], uy = s[S_UY], un = s[S_UN];
  const double ut = sqrt(1. + ux * ux + uy * uy + tau2 * un * un);
  const double uperp = sqrt(ux * ux + uy * uy), utperp = sqrt(1. + ux * ux + uy * uy);
  const double ux2 = ux * ux, uy2 = uy * uy, ut2 = ut * ut;
  if (ut * dat + ux * dax + uy * day + un * dan <= 0) return DF_OK;
  const double T = s[S_T], P = s[S_P], E = s[S_E];
  double pitt = 0, pitx = 0, pity = 0, pitn = 0, pixx = 0, pixy = 0, pixn = 0, piyy = 0, piyn = 0, pinn = 0;
  if (k.include_shear && k.df_mode == PTB) {     // pi only enters through the PTB breakdown test
    pixx = s[S_PIXX]; pixy = s[S_PIXY]; pixn = s[S_PIXN]; piyy = s[S_PIYY]; piyn = s[S_PIYN];
    pinn = (pixx * (ux2 - ut2) + piyy * (uy2 - ut2) + 2. * (pixy * ux * uy + tau2 * un * (pixn * ux + piyn * uy))) / (tau2 * utperp * utperp);
    pitn = (pixn * ux + piyn * uy + tau2 * pinn * un) / ut;
    pity = (pixy * ux + piyy * uy + tau2 * piyn * un) / ut;
    pitx = (pixx * ux + pixy * uy + tau2 * pixn * un) / ut;
    pitt = (pitx * ux + pity * uy + tau2 * pitn * un) / ut;
  }
  double bulkPi = k.include_bulk ? s[S_BULKPI] : 0.0;
  double muB = 0, Vt = 0, Vx = 0, Vy = 0, Vn = 0;
  if (k.include_baryon && k.include_diff) {
    muB = s[S_MUB]; Vx = s[S_VX]; Vy = s[S_VY]; Vn = s[S_VN];
    Vt = (Vx * ux + Vy * uy + tau2 * Vn * un) / ut;
  }
  const double Vdsigma = Vt * dat + Vx * dax + Vy * day + Vn * dan;
  if (k.df_mode == PTB) {     // :548-560
    if (bulkPi <= -P) bulkPi = -(1.0 - 1.e-5) * P;
    else if (bulkPi / P >= tb.bulk_over_P_max) bulkPi = P * (tb.bulk_over_P_max - 1.e-5);
  }
  DfCoef df;
  const int err = df_eval(tb, T, muB, E, P, bulkPi, df);
  if (err) return err;
  const Milne b = milne_basis(ut, ux, uy, un, uperp, utperp, tau);
  const double ds_time = dat * ut + dax * ux + day * uy + dan * un;          // LocalRestFrame.cpp:81-91
  const double dsx = -(dat * b.Xt + dax * b.Xx + day * b.Xy + dan * b.Xn);
  const double dsy = -(dax * b.Yx + day * b.Yy);
  const double dsz = -(dat * b.Zt + dan * b.Zn);
  const double ds_space = sqrt(dsx * dsx + dsy * dsy + dsz * dsz);
  if (k.df_mode == PTB) {
    const PiLRF pl_ = boost_pi(b, tau2, pitt, pitx, pity, pitn, pixx, pixy, pixn, piyy, piyn, pinn);
    const double shear_mod = 0.5 / df.betapi, bulk_mod = df.lambda;
    const double Axx = 1.0 + pl_.xx * shear_mod + bulk_mod, Axy = pl_.xy * shear_mod, Axz = pl_.xz * shear_mod;
    const double Ayy = 1.0 + pl_.yy * shear_mod + bulk_mod, Ayz = pl_.yz * shear_mod, Azz = 1.0 + pl_.zz * shear_mod + bulk_mod;
    const double detA = Axx * (Ayy * Azz - Ayz * Ayz) - Axy * (Axy * Azz - Ayz * Axz) + Axz * (Axy * Ayz - Ayy * Axz);
    const bool breaks = (detA <= k.deta_min || df.z < 0.0);
    *out = breaks ? ds_time * (1.0 + df.dz) * dsum[0] : ds_time * df.z * dsum[0];
  } else {
    *out = ds_time * (dsum[0] + bulkPi * dsum[1]) - ds_space * Vdsigma * dsum[2];
  }
  return DF_OK;
}

// PTM per-(cell, species) renormalisation (MomentumSpectra.cpp:790-832); NaN => species skipped.
IS3D_HD double ptm_renorm(const PrepConsts& k, const double* aux, double mass, double sign, double degeneracy, double baryon) {
  const double T = aux[0], T_mod = aux[1], alphaB = aux[2], alphaB_mod = aux[3], F = aux[4], G = aux[5];
  const double betabulk = aux[6], bulkPi = aux[7], den = aux[8];
  double renorm = 1.0;
  if (k.include_bulk) {
    const double neq_fact = T * T * T / k.two_pi2_hbarC3;
    const double dn_fact = bulkPi / betabulk, J20_fact = T * neq_fact, N10_fact = neq_fact;
    const double nmod_fact = T_mod * T_mod * T_mod / k.two_pi2_hbarC3;
    const double mbar = mass / T, mbar_mod = mass / T_mod;
    const double neq = neq_fact * degeneracy * gt_neq(k.gla_r1, k.gla_w1, k.gla_pts, mbar, alphaB, baryon, sign);
    const double N10 = baryon * N10_fact * degeneracy * gt_J10(k.gla_r1, k.gla_w1, k.gla_pts, mbar, alphaB, baryon, sign);
    const double J20 = J20_fact * degeneracy * gt_J20(k.gla_r2, k.gla_w2, k.gla_pts, mbar, alphaB, baryon, sign);
    const double n_linear = neq + dn_fact * (neq + N10 * G + J20 * F / T / T);
    const double n_mod = nmod_fact * degeneracy * gt_neq(k.gla_r1, k.gla_w1, k.gla_pts, mbar_mod, alphaB_mod, baryon, sign);
    renorm = n_linear / n_mod;
  }
  renorm /= den;
  return renorm;
}

// --- PTMA prologue part A (MomentumSpectra.cpp:1159-1285): everything up to the Newton solve.
// aniso_in: E, pl, pt, T (initial lambda), piTxx, piTxy, piTyy, WTzx, WTzy ; returns kind (0 skip)
IS3D_HD int prep_famod_a(const PrepConsts& k, const double* s, double* R, double* ain) {
  for (int f = 0; f < NREC; f++) R[f] = 0.0;
  const double tau = s[S_TAU], tau2 = tau * tau;
  const double eta = (k.dim == 3) ? s[S_ETA] : 0.0;
  const double dat = s[S_DAT], dax = s[S_DAX], day = s[S_DAY], dan = s[S_DAN];
  const double ux = s[S_UX], uy = s[S_UY], un = s[S_UN];
  const double ut = sqrt(1. + ux * ux + uy * uy + tau2 * un * un);
  if (ut * dat + ux * dax + uy * day + un * dan <= 0) { R[R_KIND] = 0.0; return 0; }
  const double ut2 = ut * ut, ux2 = ux * ux, uy2 = uy * uy;
  const double uperp = sqrt(ux * ux + uy * uy), utperp = sqrt(1. + ux * ux + uy * uy);
  const double T = s[S_T], P = s[S_P], E = s[S_E];
  const double pixx = s[S_PIXX], pixy = s[S_PIXY], pixn = s[S_PIXN], piyy = s[S_PIYY], piyn = s[S_PIYN];
  const double pinn = (pixx * (ux2 - ut2) + piyy * (uy2 - ut2) + 2. * (pixy * ux * uy + tau2 * un * (pixn * ux + piyn * uy))) / (tau2 * utperp * utperp);
  const double pitn = (pixn * ux + piyn * uy + tau2 * pinn * un) / ut;
  const double pity = (pixy * ux + piyy * uy + tau2 * piyn * un) / ut;
  const double pitx = (pixx * ux + pixy * uy + tau2 * pixn * un) / ut;
  const double pitt = (pitx * ux + pity * uy + tau2 * pitn * un) / ut;
  const double bulkPi = s[S_BULKPI];
  const double muB = k.include_baryon ? s[S_MUB] : 0.0;
  const double alphaB = muB / T;
  const Milne b = milne_basis(ut, ux, uy, un, uperp, utperp, tau);
  const PiLRF pl_ = boost_pi(b, tau2, pitt, pitx, pity, pitn, pixx, pixy, pixn, piyy, piyn, pinn);
  const double pl = P + bulkPi + pl_.zz, pt = P + bulkPi - pl_.zz / 2.;
  double piTxx = 0, piTxy = 0, piTyy = 0, WTzx = 0, WTzy = 0;
  if (k.include_shear) {
    piTxx = (pl_.xx - pl_.yy) / 2.; piTxy = pl_.xy; piTyy = -(piTxx);
    WTzx = pl_.xz; WTzy = pl_.yz;
  }
  rec_common(R, tau, eta, ut, un, ux, uy, dat, dax, day, dan, T);
  // PTMA's feq fallback has no delta-f; pi / V fields stay zero in the record
  R[R_CHEM] = alphaB; R[R_CHEMM] = alphaB;   // upsilonB = alphaB (:1292)
  // basis for the modified directions (stashed in the U/V slots until part B)
  R[R_UCX] = b.Xt; R[R_UCY] = b.Xx; R[R_UCZ] = b.Xy; R[R_USX] = b.Xn; R[R_USY] = b.Yx; R[R_USZ] = b.Yy;
  R[R_VCX] = b.Zt; R[R_VCY] = b.Zn;
  ain[0] = E; ain[1] = pl; ain[2] = pt; ain[3] = T;
  ain[4] = piTxx; ain[5] = piTxy; ain[6] = piTyy; ain[7] = WTzx; ain[8] = WTzy;
  R[R_KIND] = 2.0;
  return 1;
}

// --- PTMA prologue part B (MomentumSpectra.cpp:1372-1481), after the Newton solve.
// sol: lambda, aT, aL, broken(0/1), betapiperp, betaWperp
IS3D_HD void prep_famod_b(const PrepConsts& k, double* R, const double* ain, const double* sol, int* breakdown_out) {
  const double tau = R[R_TAU];
  const double Xt = R[R_UCX], Xx = R[R_UCY], Xy = R[R_UCZ], Xn = R[R_USX], Yx = R[R_USY], Yy = R[R_USZ];
  const double Zt = R[R_VCX], Zn = R[R_VCY];
  const double piTxx = ain[4], piTxy = ain[5], piTyy = ain[6], WTzx = ain[7], WTzy = ain[8];
  const double lambda = sol[0], aT = sol[1], aL = sol[2];
  int broken = (int)sol[3];
  const double shear_coeff = 0.5 / sol[4], diff_coeff = 1. / sol[5];
  const double Axx = aT, Ayy = aT, Azz = aL, detA = Axx * Ayy * Azz;
  const double Cxx = 1. + shear_coeff * piTxx, Cxy = shear_coeff * piTxy, Cxz = diff_coeff * WTzx * aT / (aT + aL);
  const double Cyx = Cxy, Cyy = 1. + shear_coeff * piTyy, Cyz = diff_coeff * WTzy * aT / (aT + aL);
  const double Czx = diff_coeff * WTzx * aL / (aT + aL), Czy = diff_coeff * WTzy * aL / (aT + aL), Czz = 1.;
  const double detC = Cxx * (Cyy * Czz - Cyz * Czy) - Cxy * (Cyx * Czz - Cyz * Czx) + Cxz * (Cyx * Czy - Cyy * Czx);
  const double Bxx = Axx + aT * shear_coeff * piTxx, Bxy = aT * shear_coeff * piTxy, Bxz = diff_coeff * WTzx * aT * aL / (aT + aL);
  const double Byy = Ayy + aT * shear_coeff * piTyy, Byz = diff_coeff * WTzy * aT * aL / (aT + aL), Bzz = Azz;
  const double detB = detC * detA;
  const double detB_b23 = (2. * aT + aL) * (2. * aT + aL) / 9.;
  const double B[9] = {Bxx, Bxy, Bxz, Bxy, Byy, Byz, Bxz, Byz, Bzz};
  if (detB <= k.deta_min) broken = 1;
  double eta_scale = 1;
  if (detB > k.deta_min && k.dim == 2) eta_scale = detB / detB_b23;
  const double renorm = eta_scale / detC;
  if (isnan(renorm) || isinf(renorm)) broken = 1;
  modified_directions(B, tau, Xt, Xx, Xy, Xn, Yx, Yy, Zt, Zn, R + R_UCX);
  R[R_VB] = sqrt(R[R_VCX] * R[R_VCX] + R[R_VCY] * R[R_VCY] + R[R_VCZ] * R[R_VCZ]) +
            sqrt(R[R_VSX] * R[R_VSX] + R[R_VSY] * R[R_VSY] + R[R_VSZ] * R[R_VSZ]);
  R[R_INVTM] = 1.0 / lambda;
  mod_scale_record(R);
  R[R_ETASCALE] = eta_scale; R[R_DET] = detB;
  R[R_NARROW] = (k.dim == 3 && detB < 0.01) ? 1.0 : 0.0;
  R[R_RENORM] = fabs(renorm);
  *breakdown_out = broken;
  R[R_KIND] = broken ? 1.0 : 2.0;
}

// ---------------------------------------------------------------------------
// y-terms and phi-terms
// ---------------------------------------------------------------------------
// variant flags for the separable path
enum SepFlavor : int { SEP_GRAD = 0, SEP_CE = 1, SEP_PTB = 2, SEP_FEQ = 3 };

// mode -> (separable flavour, use cosh() instead of sqrt(1+sinh^2), w_eta only on the non-eta part of p.dsigma)
IS3D_HD int sep_flavor(int mode) { return mode == GRAD ? SEP_GRAD : (mode == CE || mode == PTM) ? SEP_CE : mode == PTB ? SEP_PTB : SEP_FEQ; }
// spectra PTM/PTB: w_eta multiplies only the non-eta part of p.dsigma (MomentumSpectra.cpp:936); the
// spacetime path weights all of it (SpacetimeDistribution.cpp:1026, 1076)
IS3D_HD int quirk_pds(int mode, int op) { return (op != 0 && (mode == PTM || mode == PTB)) ? 1 : 0; }

// Species- and y-independent pieces of the separable lane coefficients, per cell (record
// fields R_S0M2 .. R_LS; see yterms / sep_setup for the factorisation).
IS3D_HD void sep_cell_consts(int mode, double* R) {
  const int fl = sep_flavor(mode);
  double s0m2 = 0.0, scb = 0.0, ssb = 0.0, l0b = 0.0, lc = 0.0, ls = 0.0;
  if (fl == SEP_GRAD) {
    s0m2 = R[R_BULK0];
    scb = -(R[R_BULK1] * R[R_UX] + R[R_DIFF0] * R[R_VX]);
    ssb = -(R[R_BULK1] * R[R_UY] + R[R_DIFF0] * R[R_VY]);
  } else if (fl == SEP_CE) {
    const double bsum = R[R_BULK0] + R[R_BULK2];
    s0m2 = -R[R_BULK2];
    scb = R[R_DIFF1] * R[R_VX]; ssb = R[R_DIFF1] * R[R_VY];
    l0b = R[R_BULK1];
    lc = -bsum * R[R_UX] - R[R_DIFF0] * R[R_VX];
    ls = -bsum * R[R_UY] - R[R_DIFF0] * R[R_VY];
  } else if (fl == SEP_PTB) {
    const double dl = R[R_DLAM] * R[R_INVT];
    s0m2 = -dl; lc = -dl * R[R_UX]; ls = -dl * R[R_UY];
  }
  R[R_S0M2] = s0m2; R[R_SCB] = scb; R[R_SSB] = ssb; R[R_L0B] = l0b; R[R_LC] = lc; R[R_LS] = ls;
}

// y-terms for (cell R, rapidity y, space-time rapidity eta, weight w).  With
// ch = cosh(y - eta), sh = sinh(y - eta), p^tau = mT ch, tau p^eta = mT sh:
//   A = ch u^tau - sh tau u^eta,  D = w (ch dsigma_tau + sh dsigma_eta/tau)   (:304-330)
//   Q1 = pi^tt ch^2 + tau^2 pi^ee sh^2 - 2 tau pi^te ch sh,  W = V^t ch - tau V^e sh
// and the separable delta-f coefficients factor as  S0 = mT^2 S2 + mT b S1 + m^2 R_S0M2,
// Sc = mT SC1 + b R_SCB,  Ss = mT SS1 + b R_SSB,  L0 = mT L1 + b R_L0B  (see sep_setup).
// mu_slots = false: rows of kYRowLY doubles (k_spectra's per-lane rows), without Y_MU2 / Y_MU (mod_setup
// then takes |sig U| itself, ymu = false)
IS3D_HD void yterms(int mode, int op, const double* R, double y, double eta, double w, double* Y, bool mu_slots = true,
                    bool mod_only = false) {
  const int quirk = quirk_pds(mode, op);
  if (mode >= PTM && mod_only) {
    // the modified launches' rows (k_spectra / k_dndx MODMAIN): their lanes read the modified slots, Y_WDX / Y_WDY,
    // Y_NARROW and Y_W only --
    // the separable slots serve the F_FB launch, which builds its own rows
    const double es = R[R_ETASCALE];
    double shm, chm;
    sinh_cosh(y - es * eta, &shm, &chm);
    const double ux = chm * R[R_UCX] + shm * R[R_USX];
    const double uy = chm * R[R_UCY] + shm * R[R_USY];
    const double uz = chm * R[R_UCZ] + shm * R[R_USZ];
    Y[Y_MUX] = ux; Y[Y_MUY] = uy; Y[Y_MUZ] = uz;
    Y[Y_MD] = quirk ? (w * chm * R[R_DAT] + shm * R[R_DANT]) : w * (chm * R[R_DAT] + shm * R[R_DANT]);
    Y[Y_WDX] = w * R[R_DAX]; Y[Y_WDY] = w * R[R_DAY];        // the lane forms' p.dsigma (k_dndx, mod_setup Dc / Ds)
    Y[Y_NARROW] = (R[R_NARROW] != 0.0 && fabs(y - eta) < R[R_DET]) ? 1.0 : 0.0;
    if (mu_slots) {
      Y[Y_MU2] = fma(ux, ux, fma(uy, uy, uz * uz));
      Y[Y_MU] = sqrt(Y[Y_MU2]);
    }
    Y[Y_W] = w;
    return;
  }
  // separable part: p^tau = mT cosh(y-eta) (spectra Grad/CE: sqrt(1+sinh^2), MomentumSpectra.cpp:307-308;
  // the spacetime path uses cosh, SpacetimeDistribution.cpp:313)
  double sh, chx;
  sinh_cosh(y - eta, &sh, &chx);
  const double ch = (mode <= CE && op != 0) ? sqrt(1.0 + sh * sh) : chx;
  const double A = ch * R[R_UT] - sh * R[R_TAUUN];
  Y[Y_A] = A;
  Y[Y_AT] = A * R[R_INVT];
  Y[Y_D] = quirk ? (w * ch * R[R_DAT] + sh * R[R_DANT]) : w * (ch * R[R_DAT] + sh * R[R_DANT]);
  Y[Y_WDX] = w * R[R_DAX]; Y[Y_WDY] = w * R[R_DAY];
  const double shear = R[R_SHEAR];
  const double Q1 = R[R_PITT] * ch * ch + R[R_T2PINN] * sh * sh - 2.0 * R[R_TPITN] * ch * sh;
  const double W = R[R_VT] * ch - R[R_TVN] * sh;
  // shear p.pi.p linear part: (pc, ps) . 2 shear mT (sh tau pi^{n i} - ch pi^{t i})
  const double Pc = 2.0 * shear * (sh * R[R_TPIXN] - ch * R[R_PITX]);
  const double Ps = 2.0 * shear * (sh * R[R_TPIYN] - ch * R[R_PITY]);
  const int fl = sep_flavor(mode);
  double S2 = shear * Q1, S1 = 0.0, SC1 = Pc, SS1 = Ps, L1 = 0.0;
  if (fl == SEP_GRAD) {
    const double bulk2 = R[R_BULK2], diff1 = R[R_DIFF1];
    S2 = (bulk2 * A + diff1 * W) * A + shear * Q1;
    S1 = R[R_BULK1] * A + R[R_DIFF0] * W;
    SC1 = Pc - (2.0 * bulk2 * A + diff1 * W) * R[R_UX] - diff1 * A * R[R_VX];
    SS1 = Ps - (2.0 * bulk2 * A + diff1 * W) * R[R_UY] - diff1 * A * R[R_VY];
  } else if (fl == SEP_CE) {
    S1 = -R[R_DIFF1] * W;
    L1 = (R[R_BULK0] + R[R_BULK2]) * A + R[R_DIFF0] * W;
  } else if (fl == SEP_PTB) {
    L1 = R[R_DLAM] * R[R_INVT] * A;
  }
  Y[Y_S2] = S2; Y[Y_S1] = S1; Y[Y_SC1] = SC1; Y[Y_SS1] = SS1; Y[Y_L1] = L1;
  if (mode >= PTM) {
    const double es = R[R_ETASCALE];
    double shm, chm;
    sinh_cosh(y - es * eta, &shm, &chm);
    Y[Y_MUX] = chm * R[R_UCX] + shm * R[R_USX];
    Y[Y_MUY] = chm * R[R_UCY] + shm * R[R_USY];
    Y[Y_MUZ] = chm * R[R_UCZ] + shm * R[R_USZ];
    Y[Y_MD] = quirk ? (w * chm * R[R_DAT] + shm * R[R_DANT]) : w * (chm * R[R_DAT] + shm * R[R_DANT]);
    Y[Y_NARROW] = (R[R_NARROW] != 0.0 && fabs(y - eta) < R[R_DET]) ? 1.0 : 0.0;
    // |sig U|^2 and |sig U| once per (cell, q) instead of once per (cell, lane) in mod_setup
    if (mu_slots) {
      const double ux = Y[Y_MUX], uy = Y[Y_MUY], uz = Y[Y_MUZ];
      Y[Y_MU2] = fma(ux, ux, fma(uy, uy, uz * uz));
      Y[Y_MU] = sqrt(Y[Y_MU2]);
    }
  } else {
    Y[Y_MUX] = Y[Y_MUY] = Y[Y_MUZ] = Y[Y_MD] = Y[Y_NARROW] = 0.0;
    if (mu_slots) Y[Y_MU2] = Y[Y_MU] = 0.0;
  }
  Y[Y_W] = w;                      // w_eta (PD-table scale, sep_setup)
}

// phi-terms.  Everything the integrand needs per (cell, phi) except two numbers is linear in
// (pc, ps) = (pT cos phi, pT sin phi): u.p, p.dsigma, pi^{t i} p_i, pi^{n i} p_i, V.p and the
// modified momentum A^{-1} p all are.  Those linear pieces are folded into per-lane
// coefficients at sep_setup / mod_setup time, so a point reads only
//   cs = {pc, ps}        per phi          (shared by every cell of the workgroup)
//   bp = {b', Phi}       per (cell, phi)  b' = exp(pT B/T - zb) with B = u^x cos + u^y sin and
//                                         zb = pT |u_perp|/T its bound over phi (so b' <= 1),
//                                         Phi = the part of delta-f quadratic in (pc, ps)
// Grad: Phi = shear p_i pi^{ij} p_j + bulk2 (pT B)^2 + c4 (pT B)(V.p)   (E^2 and E (V.p) cross terms)
// CE / PTM / PTB (separable): Phi = shear p_i pi^{ij} p_j
IS3D_HD dbl2 phiterms(int mode, const double* R, double pT, double c, double s, const double* etab) {
  const double PTB = pT * (c * R[R_UX] + s * R[R_UY]);
  const double Q3 = R[R_SHEAR] * (pT * pT * (R[R_PIXX] * c * c + R[R_PIYY] * s * s + 2.0 * R[R_PIXY] * c * s));
  dbl2 o;
  // b' e^-zb <= 1, zb = pT |u_perp| / T >= pT B / T (table exp; underflows to 0 below e^-745)
  o.x = exp_tab(exp_tab_coef(), etab, fma(PTB, R[R_INVT], -pT * R[R_ZB]) * kInvLn2xN);
  if (mode == GRAD) {
    const double WP = pT * (R[R_VX] * c + R[R_VY] * s);
    o.y = Q3 + PTB * (R[R_BULK2] * PTB + R[R_DIFF1] * WP);
  } else {
    o.y = Q3;
  }
  return o;
}

// exp(x) overflows above this; 1/(inf + sign) == 0 exactly as in the reference
static constexpr double kExpMax = 709.782712893384;

// ---------------------------------------------------------------------------
// Lane state for one (cell, species, pT, q) and the per-phi integrand.
// ---------------------------------------------------------------------------
// A lin3 is c0 + cc pc + cs ps.
struct SepLane {
  double a, ssc, sign;         // a = exp(mT A/T - chem - zb - S), ssc = sign e^-S:  b' / (a + ssc b') = e^S feq
  double D0, Dc, Ds;           // e^-S p.dsigma (x w_eta)
  double S0, Sc, Ss;           // Grad: S (with Phi); CE/PTB: numerator N of the 1/E part (with Phi)
  double E0, Ec, Es;           // CE/PTB: E = u.p
  double L0, Lc, Ls;           // CE/PTB: part of delta-f linear in E
  double c0;                   // PTB: constant added outside (1 - sign feq)
  double x, Zc, Zs;            // slow path: feq = 1/(exp(x - Zc pc - Zs ps) + sign)
  int skip, fast;
  int tail;                    // Boltzmann tail (sep_setup, allow_tail): a + ssc b' == a at every phi point
  int near;                    // near the tail (sep_setup, allow_near): ssc b' / a <= e^-kNearX at every phi point
  double escw;                 // 2^-k w_eta (PD-table scale)
};

// Boltzmann-tail bound: for an exponent x >= kTailX, e^-x < 2^-54, so exp(x) + sign == exp(x) and
// 1 - sign f_eq == 1 in FP64 exactly (the sum rounds back to the larger term); a lane whose smallest
// exponent over phi exceeds it needs no per-point reciprocal at all
static constexpr double kTailX = 37.5;
// fast-path domain of sep_setup: smallest exponent x - zb >= kExpFast (sep_slow_cell bounds it per cell)
static constexpr double kExpFast = -300.0;
// near-tail bound: for an exponent x >= kNearX, u = sign e^-x <= 1.6e-8, so 1 / (1 + u) = 1 - u to u^2 <= 2.4e-16
// (the rounding of the reciprocal it replaces: rcp1, ~2e-15); a Grad lane whose smallest exponent exceeds it
// takes (1 - u) (1 + (1 - u) S) = (1 + S) - u (1 + 2 S) per point, no reciprocal (sep_quad_tb_near_t)
static constexpr double kNearX = 18.0;
// IS3D_SEP_INVA: sep_setup's default for inv_a (tail / near lanes take 1/a from one table exp of -xs instead of a and
// its reciprocal).  MI355X (profiles/round6_r6e_ab_inva.log): config 2 operation 0 Grad k_dndx 319.6 -> 313.0 ms, but
// the F_TS Grad k_spectra 151.0 -> 155.7 ms (same VGPRs, more SGPR spills) -- so off by default, on in k_dndx
#ifndef IS3D_SEP_INVA
#define IS3D_SEP_INVA 0
#endif

// 1/d for finite normal d: v_rcp_f64 (measured max rel. error 4.5e-8 on gfx950) + one
// Newton step (~2e-15); IEEE division on the host.  Callers guarantee d is finite.
IS3D_HD double rcp1(double d) {
#if defined(__HIP_DEVICE_COMPILE__)
  const double r = __builtin_amdgcn_rcp(d);
  return fma(r, fma(-d, r, 1.0), r);
#else
  return 1.0 / d;
#endif
}

// Per-(cell, q, species) setup for the separable integrand.  Returns skip=1 when every
// phi point underflows (exp argument > 709.78 for all phi: contributes exactly 0).
// The delta-f polynomials (MomentumSpectra.cpp:304-361 Grad, :565-600 CE, :920-923 PTB) are
// expanded in (pc, ps); their coefficients factor into (cell, y) terms (yterms), per-cell
// terms (sep_cell_consts) and the lane's mT, m^2, baryon number b:
//   Grad  S  = S0 + Phi + Sc pc + Ss ps               delta-f = (1 - sign feq) S
//   CE    S  = (S0 + Phi + Sc pc + Ss ps) / E + L0 + Lc pc + Ls ps,   E = mT A - ux pc - uy ps
//   PTB   as CE, delta-f = (1 - sign feq) S + dz - 3 dlambda
// mT2 = mT * mT and mTb = mT * b are per-lane constants hoisted by the caller.
//
// allow_tail (callers with a tail loop, sep_quad_tb_tail_t; 2 = decided per wavefront on the device): lanes
// whose smallest exponent xs = x - zb
// exceeds kTailX get tail = 1; their den = a + ssc b' equals a for every phi (kTailX), so f_eq = b'/a and
// 1 - sign f_eq = 1 exactly, and the lane keeps the delta-f coefficients unscaled (sa = 1) and 1/a
// folded into the p.dsigma coefficients D0, Dc, Ds, escw: a point is (w p.dsigma f_eq)(1 + delta-f)
// with no reciprocal (Grad: 5 VALU ops instead of 12).
// sep_setup's skip test alone (the same two operations): callers test it first, so a wavefront whose lanes all
// skip the cell branches past the lane setup (~65 instructions) instead of computing it
IS3D_HD bool sep_skips(const double* R, const double* Y, double mT, double pT, double baryon) {
  return fma(mT, Y[Y_AT], -baryon * R[R_CHEM]) - pT * R[R_ZB] > kExpMax;
}

// Can a lane of this cell leave sep_setup's fast path (smallest exponent x - zb below -300)?  With
// A(y - eta) = ch u^tau - sh tau u^eta >= A_min = sqrt(u^tau^2 - (tau u^eta)^2) (its minimum over all rapidities)
// and zb = pT |u_perp| / T, x - zb = (mT A - pT |u_perp|) / T - b chem >= min(0, pT_max (A_min - |u_perp|)) / T
// - b_max |chem| (mT >= pT); for a normalised u, A_min = sqrt(1 + u_perp^2) > |u_perp| and the bound is
// -b_max |chem|: such lanes need |mu_B| / T > ~300.  Conservative (a margin of 10), NaN-safe.
IS3D_HD bool sep_slow_cell(const double* R, double pT_max, double b_max) {
  const double a2 = R[R_UT] * R[R_UT] - R[R_TAUUN] * R[R_TAUUN];
  const double amin = a2 > 0.0 ? sqrt(a2) : 0.0, up = sqrt(R[R_UX] * R[R_UX] + R[R_UY] * R[R_UY]);
  const double lb = fmin(0.0, pT_max * (amin - up)) * R[R_INVT] - b_max * fabs(R[R_CHEM]);
  return !(lb > kExpFast + 10.0);
}

IS3D_HD void sep_setup(int flavor, const double* R, const double* Y, double mT, double mT2, double m2, double mTb,
                       double pT, double sign, double baryon, const double* etab, SepLane& L, int allow_tail = 0,
                       int allow_near = 0, bool inv_a = IS3D_SEP_INVA) {
  L.sign = sign;
  L.x = fma(mT, Y[Y_AT], -baryon * R[R_CHEM]);
  const double zb = pT * R[R_ZB];                 // >= max_j |pT B_j / T|
  L.skip = (L.x - zb > kExpMax) ? 1 : 0;
  // b' carries e^-zb, so a = e^(x - zb) 2^-k.  u.p > 0 makes x - zb >= -chem, so without the
  // shift the lane's a spans [e^-chem, e^710]; for x - zb > 150 the exact scale esc = 2^-k with
  // k = floor((x - zb - 150) / ln2) keeps every denominator a + ssc b' in ~[1e-2, e^151] (times
  // E = u.p < e^10 for CE/PTB), so the product of four of them (one reciprocal per four points,
  // sep_quad_t) stays finite and normal.  The scale is exact, so
  // a = e^(x - zb) 2^-k is as accurate as e^(x - zb) itself (table exp, ~1 ulp)
  const double xs = L.x - zb;
  L.fast = (xs >= kExpFast) ? 1 : 0;
  L.tail = (allow_tail && xs > kTailX) ? 1 : 0;
#if defined(__HIP_DEVICE_COMPILE__)
  // allow_tail == 2: one decision per wavefront (all its live lanes in the tail, or none), so a wavefront
  // whose lanes straddle the tail bound runs the normal fours only instead of both phi loops back to back
  // (the vote is passed through a VGPR: as a wave-uniform SGPR value it made the compiler restructure the
  // lane loops and spill 97 VGPRs)
  if (allow_tail == 2) {
    int t = __all(L.tail);
    asm volatile("" : "+v"(t));
    L.tail = t;
  }
#endif
  // allow_near (with allow_tail; 2 = per wavefront on the device, as the tail vote): near-tail lanes
  L.near = (allow_near && !L.tail && xs > kNearX) ? 1 : 0;
#if defined(__HIP_DEVICE_COMPILE__)
  if (allow_near == 2) {
    int t = __all(xs > kNearX) && !L.tail;
    asm volatile("" : "+v"(t));
    L.near = t;
  }
#endif
  const int k = (L.fast && xs > 150.0) ? (int)((xs - 150.0) * 1.4426950408889634) : 0;
  // tail and near lanes (xs > kNearX, so fast) use only 1/a = e^-xs 2^k: one table exp of -xs instead of a = e^xs 2^-k
  // and its reciprocal (IS3D_SEP_INVA; a is left 0, none of their loops reads it)
  const bool inva = inv_a && (L.tail || L.near);
  double ra = 0.0;
  if (inva) {
    ra = exp_tab(exp_tab_coef(), etab, -xs * kInvLn2xN, -k);
    L.a = 0.0;
  } else {
    L.a = L.fast ? exp_tab(exp_tab_coef(), etab, xs * kInvLn2xN, k) : 0.0;
  }
  const double esc = ldexp(1.0, -k);
  L.ssc = sign * esc;
  L.escw = esc * Y[Y_W];
  if (!L.fast) { L.Zc = R[R_UX] * R[R_INVT]; L.Zs = R[R_UY] * R[R_INVT]; } else { L.Zc = L.Zs = 0.0; }
  L.D0 = esc * (mT * Y[Y_D]); L.Dc = esc * Y[Y_WDX]; L.Ds = esc * Y[Y_WDY];
  // fast lanes carry the delta-f coefficients pre-multiplied by a (see sep_fast_tail)
  const double sa = (L.fast && !L.tail && !L.near) ? L.a : 1.0;
  L.S0 = sa * fma(mT2, Y[Y_S2], fma(mTb, Y[Y_S1], m2 * R[R_S0M2]));
  L.Sc = sa * fma(mT, Y[Y_SC1], baryon * R[R_SCB]);
  L.Ss = sa * fma(mT, Y[Y_SS1], baryon * R[R_SSB]);
  L.E0 = mT * Y[Y_A]; L.Ec = -R[R_UX]; L.Es = -R[R_UY];
  L.L0 = sa * fma(mT, Y[Y_L1], baryon * R[R_L0B]); L.Lc = sa * R[R_LC]; L.Ls = sa * R[R_LS];
  L.c0 = (flavor == SEP_PTB) ? R[R_DZ] - 3.0 * R[R_DLAM] : 0.0;
  if (L.tail || L.near) {   // f_eq = b' / a: fold 1/a into the p.dsigma coefficients (both carry the same 2^-k)
    if (!inva) ra = rcp1(L.a);
    L.D0 *= ra; L.Dc *= ra; L.Ds *= ra; L.escw *= ra;
    if (L.near) L.ssc *= ra;         // u = ssc b' (sep_quad_tb_near_t)
  }
}

IS3D_HD double lin(double c0, double cc, double cs, dbl2 p) { return fma(cc, p.x, fma(cs, p.y, c0)); }

// fma(a, b, c) with c wave-uniform in an SGPR (an F_TS table operand, kernels.h): one VOP3 v_fma_f64.  Left to
// the compiler, fma(vgpr, vgpr, sgpr) became v_fmac_f64 on a VGPR copy of c -- two v_mov_b32 per point
IS3D_HD double fma_vvs(double a, double b, double c) {
#if defined(__HIP_DEVICE_COMPILE__)
  double r;
  asm("v_fma_f64 %0, %1, %2, %3" : "=v"(r) : "v"(a), "v"(b), "s"(c));
  return r;
#else
  return fma(a, b, c);
#endif
}

// Slow-path tail (per-point exp, unscaled coefficients): returns w * p.dsigma * f_eq (1 + delta-f)
// (0 when outflow-cut), with 1 - sign f_eq and 1/E formed as in the reference.
template <int FL, bool REG, bool OUT>
IS3D_HD double sep_tail(const SepLane& L, dbl2 cs, dbl2 bp, double pds, double feq, double iE) {
  const bool needE = (FL == SEP_CE || FL == SEP_PTB);
  double g = feq * pds;
  if (OUT) g = (pds <= 0.0) ? 0.0 : g;
  if (FL == SEP_FEQ) return g;
  const double fbar = fma(-L.sign, feq, 1.0);
  double S = fma(L.Sc, cs.x, fma(L.Ss, cs.y, L.S0 + bp.y));
  if (needE) S = fma(S, iE, lin(L.L0, L.Lc, L.Ls, cs));
  double t;
  if (REG) {
    double dfv = fbar * S;
    if (FL == SEP_PTB) dfv += L.c0;
    t = 1.0 + fmax(-1.0, fmin(dfv, 1.0));
  } else {
    t = fma(fbar, S, (FL == SEP_PTB) ? 1.0 + L.c0 : 1.0);
  }
  return g * t;
}

// Fast-path tail.  With den = a + ssc b' and rq = 1/(den E) (CE/PTB; 1/den for Grad/f_eq):
//   e^S f_eq = b' E rq,   1 - sign f_eq = 1 - ssc e^S f_eq = a / den = a E rq   (exactly),
// so f_eq (1 + delta-f) = b' E rq (1 + rq (S' + E L'))   [CE/PTB: delta-f = (1 - sign f_eq)(S/E + L)]
//                         b' rq (1 + rq S')              [Grad:   delta-f = (1 - sign f_eq) S]
// with S' = a S, L' = a L (sep_setup folds a into the lane coefficients, a Phi is one FMA here).
// 1 - sign f_eq becomes a / den instead of 1 - sign f_eq: the same number without the
// reference's cancellation for bosons near f_eq = 1 (differences at the 1e-16 absolute level).
template <int FL, bool REG, bool OUT>
IS3D_HD double sep_fast_tail(const SepLane& L, dbl2 cs, dbl2 bp, double pds, double E, double rq) {
  const bool needE = (FL == SEP_CE || FL == SEP_PTB);
  const double pb = pds * bp.x;
  const double w = needE ? pb * (E * rq) : pb * rq;     // w_eta p.dsigma f_eq
  double g;
  if (FL == SEP_FEQ) {
    g = w;
  } else {
    double in = fma(L.a, bp.y, lin(L.S0, L.Sc, L.Ss, cs));
    if (needE) in = fma(E, lin(L.L0, L.Lc, L.Ls, cs), in);
    double t;
    if (REG) {
      double dfv = rq * in;
      if (FL == SEP_PTB) dfv += L.c0;
      t = 1.0 + fmax(-1.0, fmin(dfv, 1.0));
    } else {
      t = fma(rq, in, (FL == SEP_PTB) ? 1.0 + L.c0 : 1.0);
    }
    g = w * t;
  }
  return (OUT && pds <= 0.0) ? 0.0 : g;
}

// phi points per lane: the block size among 32, 24, 8, 2 that minimises the padded points plus the
// per-lane setup (~60 VALU ops, ~4.5 points' worth) of every block; ties to the larger block:
// 1 -> 2, 16 -> 8, 24 / 48 -> 24, 32 -> 32, 100 -> 24
IS3D_HD int spectra_kj(int nphi) {
  const int cand[4] = {32, 24, 8, 2};
  int best = 32;
  double best_cost = 1e300;
  for (int kj : cand) {
    const long nb = (nphi + kj - 1) / kj;
    const double cost = (double)(nb * kj) + 4.5 * (double)nb;
    if (cost < best_cost) { best = kj; best_cost = cost; }
  }
  return best;
}

// spectra_kj with lane fill: k_spectra runs lanes x ceil(nphi / KJ) tasks per pT in 256-lane workgroups,
// so for few (species x q) lanes (pikp 2+1D: 3 x 24 = 72) a 24-point block leaves 72% of a workgroup
// idle and a smaller block fills it: cost = lane slots actually launched x (KJ + the 4.5-point setup)
IS3D_HD int spectra_kj_fill(int nphi, long lanes) {
  const int cand[4] = {32, 24, 8, 2};
  int best = 32;
  double best_cost = 1e300;
  for (int kj : cand) {
    const long nb = (nphi + kj - 1) / kj;
    const long slots = (lanes * nb + 255) / 256 * 256;
    const double cost = (double)slots * ((double)kj + 4.5);
    if (cost < best_cost) { best = kj; best_cost = cost; }
  }
  return best;
}

// Fast separable lanes take their phi points four per reciprocal (sep_quad_t) when the phi block is a
// multiple of 4, pairs otherwise (MI355X A/B: RTA-CE +5.5%, profiles/round1_r1q_ab_quad.log; Grad +1.2%
// without prefetch while it spilled, round1_r1t_ab_gq.log, +1.2% more with it once spill-free, round1_r1w_ab_gpf.log)
IS3D_HD bool sep_quads(int mode, int kj) { return kj % 4 == 0; }

// One separable integrand point; returns w * p.dsigma * f (0 when outflow-cut).
// FL: separable flavour; REG: regulate_deltaf; OUT: outflow; FAST: exp factorised (see sep_setup).
template <int FL, bool REG, bool OUT, bool FAST>
IS3D_HD double sep_point_t(const SepLane& L, dbl2 cs, dbl2 bp) {
  const double pds = lin(L.D0, L.Dc, L.Ds, cs);
  const bool needE = (FL == SEP_CE || FL == SEP_PTB);
  const double E = needE ? lin(L.E0, L.Ec, L.Es, cs) : 1.0;
  if (FAST) {
    const double den = fma(L.ssc, bp.x, L.a);
    return sep_fast_tail<FL, REG, OUT>(L, cs, bp, pds, E, rcp1(needE ? den * E : den));
  }
  // feq = 1/(exp(u.p/T - chem) + sign)
  const double feq = 1.0 / (exp(L.x - lin(0.0, L.Zc, L.Zs, cs)) + L.sign);
  return sep_tail<FL, REG, OUT>(L, cs, bp, pds, feq, needE ? 1.0 / E : 0.0);
}

// Two fast-path points of one lane with one reciprocal: 1/q0 = q1/(q0 q1), 1/q1 = q0/(q0 q1),
// q = a + ssc b' (times E for CE/PTB).  sep_setup bounds every q to ~[1e-3, e^310], so
// q0 q1 is finite and normal.
template <int FL, bool REG, bool OUT>
IS3D_HD void sep_pair_t(const SepLane& L, dbl2 c0, dbl2 b0, dbl2 c1, dbl2 b1, double& v0, double& v1) {
  const bool needE = (FL == SEP_CE || FL == SEP_PTB);
  const double pds0 = lin(L.D0, L.Dc, L.Ds, c0), pds1 = lin(L.D0, L.Dc, L.Ds, c1);
  const double den0 = fma(L.ssc, b0.x, L.a), den1 = fma(L.ssc, b1.x, L.a);
  const double E0 = needE ? lin(L.E0, L.Ec, L.Es, c0) : 1.0, E1 = needE ? lin(L.E0, L.Ec, L.Es, c1) : 1.0;
  const double q0 = needE ? den0 * E0 : den0, q1 = needE ? den1 * E1 : den1;
  const double r = rcp1(q0 * q1);
  v0 = sep_fast_tail<FL, REG, OUT>(L, c0, b0, pds0, E0, r * q1);
  v1 = sep_fast_tail<FL, REG, OUT>(L, c1, b1, pds1, E1, r * q0);
}

// Two Boltzmann-tail points (sep_setup allow_tail: 1/a folded into D0 / Dc / Ds, delta-f coefficients
// unscaled; k_dndx's pairs): pb = w p.dsigma f_eq = lin(D0, Dc, Ds) b', then as sep_quad_pd_tail_t
//   Grad  pb (1 + S)        RTA-CE  pb (1 + L + S / E), one 1/E per pair
template <int FL, bool REG, bool OUT>
IS3D_HD void sep_pair_tail_t(const SepLane& L, dbl2 c0, dbl2 b0, dbl2 c1, dbl2 b1, double& v0, double& v1) {
  constexpr bool needE = FL == SEP_CE;
  double rE0 = 0.0, rE1 = 0.0;
  if (needE) {
    const double E0 = lin(L.E0, L.Ec, L.Es, c0), E1 = lin(L.E0, L.Ec, L.Es, c1);
    const double r = rcp1(E0 * E1);
    rE0 = r * E1; rE1 = r * E0;
  }
  const dbl2 c[2] = {c0, c1}, b[2] = {b0, b1};
  const double rE[2] = {rE0, rE1};
  double v[2];
#pragma unroll
  for (int i = 0; i < 2; i++) {
    double pb = lin(L.D0, L.Dc, L.Ds, c[i]) * b[i].x;
    if (OUT) pb = (pb <= 0.0) ? 0.0 : pb;
    const double S = lin(L.S0, L.Sc, L.Ss, c[i]) + b[i].y;
    const double dfv = needE ? fma(S, rE[i], lin(L.L0, L.Lc, L.Ls, c[i])) : S;
    const double t = REG ? 1.0 + fmax(-1.0, fmin(dfv, 1.0)) : 1.0 + dfv;
    v[i] = pb * t;
  }
  v0 = v[0]; v1 = v[1];
}

// Four fast-path points with one reciprocal: r = 1/(q0 q1 q2 q3), 1/(q0 q1) = r q2 q3, then as the pair
template <int FL, bool REG, bool OUT>
IS3D_HD void sep_quad_t(const SepLane& L, const dbl2* c, const dbl2* b, double* v) {
  const bool needE = (FL == SEP_CE || FL == SEP_PTB);
  double pds[4], E[4], q[4];
#pragma unroll
  for (int i = 0; i < 4; i++) {
    pds[i] = lin(L.D0, L.Dc, L.Ds, c[i]);
    const double den = fma(L.ssc, b[i].x, L.a);
    E[i] = needE ? lin(L.E0, L.Ec, L.Es, c[i]) : 1.0;
    q[i] = needE ? den * E[i] : den;
  }
  const double q01 = q[0] * q[1], q23 = q[2] * q[3];
  const double r = rcp1(q01 * q23);
  const double r01 = r * q23, r23 = r * q01;
  v[0] = sep_fast_tail<FL, REG, OUT>(L, c[0], b[0], pds[0], E[0], r01 * q[1]);
  v[1] = sep_fast_tail<FL, REG, OUT>(L, c[1], b[1], pds[1], E[1], r01 * q[0]);
  v[2] = sep_fast_tail<FL, REG, OUT>(L, c[2], b[2], pds[2], E[2], r23 * q[3]);
  v[3] = sep_fast_tail<FL, REG, OUT>(L, c[3], b[3], pds[3], E[3], r23 * q[2]);
}

IS3D_HD void sep_pair(int flavor, const SepLane& L, dbl2 c0, dbl2 b0, dbl2 c1, dbl2 b1, int regulate, int outflow,
                      double& v0, double& v1) {
#define IS3D_PAIR_CASE(FLV)                                                                       \
  if (flavor == FLV) {                                                                            \
    if (regulate) {                                                                               \
      if (outflow) sep_pair_t<FLV, true, true>(L, c0, b0, c1, b1, v0, v1);                        \
      else sep_pair_t<FLV, true, false>(L, c0, b0, c1, b1, v0, v1);                               \
    } else {                                                                                      \
      if (outflow) sep_pair_t<FLV, false, true>(L, c0, b0, c1, b1, v0, v1);                       \
      else sep_pair_t<FLV, false, false>(L, c0, b0, c1, b1, v0, v1);                              \
    }                                                                                             \
    return;                                                                                       \
  }
  IS3D_PAIR_CASE(SEP_GRAD)
  IS3D_PAIR_CASE(SEP_CE)
  IS3D_PAIR_CASE(SEP_PTB)
  IS3D_PAIR_CASE(SEP_FEQ)
#undef IS3D_PAIR_CASE
}

// p.dsigma b' table.  p.dsigma = mT Y_D + w_eta (dsigma_x pc + dsigma_y ps) (Y_D carries w_eta), so with
//   PD = (dsigma_x pc + dsigma_y ps) b'        per (cell, phi), shared by every lane of the workgroup
// a fast lane gets e^-S w p.dsigma b' = fma(D0, b', escw PD) (escw = 2^-k w_eta; D0 = 2^-k mT Y_D) in
// two ops instead of two FMAs for p.dsigma and a multiply by b' (SC = false: a caller that knows
// escw == 1 for the whole wave, one op).  The outflow cut tests p.dsigma b' <= 0: the same sign as
// p.dsigma for b' > 0, and the point is 0 anyway at b' = 0.
IS3D_HD double sep_pd(const double* R, dbl2 cs, double bpx) { return fma(R[R_DAX], cs.x, R[R_DAY] * cs.y) * bpx; }

// sep_fast_tail with pb = p.dsigma b' given
template <int FL, bool REG, bool OUT>
IS3D_HD double sep_fast_tail_pb(const SepLane& L, dbl2 cs, dbl2 bp, double pb, double E, double rq) {
  const bool needE = (FL == SEP_CE || FL == SEP_PTB);
  const double w = needE ? pb * (E * rq) : pb * rq;
  double g;
  if (FL == SEP_FEQ) {
    g = w;
  } else {
    double in = fma(L.a, bp.y, lin(L.S0, L.Sc, L.Ss, cs));
    if (needE) in = fma(E, lin(L.L0, L.Lc, L.Ls, cs), in);
    double t;
    if (REG) {
      double dfv = rq * in;
      if (FL == SEP_PTB) dfv += L.c0;
      t = 1.0 + fmax(-1.0, fmin(dfv, 1.0));
    } else {
      t = fma(rq, in, (FL == SEP_PTB) ? 1.0 + L.c0 : 1.0);
    }
    g = w * t;
  }
  return (OUT && pb <= 0.0) ? 0.0 : g;
}

// sep_quad_t with p.dsigma b' from the PD table (pd[i] = sep_pd of point i; SC: scale by escw)
template <int FL, bool REG, bool OUT, bool SC = false>
IS3D_HD void sep_quad_pd_t(const SepLane& L, const dbl2* c, const dbl2* b, const double* pd, double* v) {
  const bool needE = (FL == SEP_CE || FL == SEP_PTB);
  double pb[4], E[4], q[4];
#pragma unroll
  for (int i = 0; i < 4; i++) {
    pb[i] = fma(L.D0, b[i].x, SC ? L.escw * pd[i] : pd[i]);
    const double den = fma(L.ssc, b[i].x, L.a);
    E[i] = needE ? lin(L.E0, L.Ec, L.Es, c[i]) : 1.0;
    q[i] = needE ? den * E[i] : den;
  }
  const double q01 = q[0] * q[1], q23 = q[2] * q[3];
  const double r = rcp1(q01 * q23);
  const double r01 = r * q23, r23 = r * q01;
  v[0] = sep_fast_tail_pb<FL, REG, OUT>(L, c[0], b[0], pb[0], E[0], r01 * q[1]);
  v[1] = sep_fast_tail_pb<FL, REG, OUT>(L, c[1], b[1], pb[1], E[1], r01 * q[0]);
  v[2] = sep_fast_tail_pb<FL, REG, OUT>(L, c[2], b[2], pb[2], E[2], r23 * q[3]);
  v[3] = sep_fast_tail_pb<FL, REG, OUT>(L, c[3], b[3], pb[3], E[3], r23 * q[2]);
}

// RTA-CE fours of the per-lane launch with the cell's {TE, T2} table as well (pe[i], as in sep_quad_tb_t):
// E = E0 + TE and the lane's linear delta-f part a (L0/a + Lc pc + Ls ps) = fma(a, T2, L0) -- two ops per point
// fewer than the lane's own linear forms.  TAIL: a Boltzmann-tail lane (sep_setup allow_tail: unscaled
// coefficients, 1/a in p.dsigma), acc += pb (1 + L0 + T2 + S / E), one 1/E per four points.
template <bool REG, bool OUT, bool TAIL>
IS3D_HD void sep_quad_pde_t(const SepLane& L, const dbl2* c, const dbl2* b, const double* pd, const dbl2* pe,
                            double* acc) {
  double pb[4], E[4], q[4];
#pragma unroll
  for (int i = 0; i < 4; i++) {
    pb[i] = fma(L.D0, b[i].x, L.escw * pd[i]);
    E[i] = L.E0 + pe[i].x;
    q[i] = TAIL ? E[i] : fma(L.ssc, b[i].x, L.a) * E[i];
  }
  const double q01 = q[0] * q[1], q23 = q[2] * q[3];
  const double r = rcp1(q01 * q23);
  const double r01 = r * q23, r23 = r * q01;
  const double rq[4] = {r01 * q[1], r01 * q[0], r23 * q[3], r23 * q[2]};
#pragma unroll
  for (int i = 0; i < 4; i++) {
    if (TAIL) {   // rq = 1/E
      double p = pb[i];
      if (OUT) p = (p <= 0.0) ? 0.0 : p;
      const double S = lin(L.S0, L.Sc, L.Ss, c[i]) + b[i].y;
      double t;
      if (REG) t = 1.0 + fmax(-1.0, fmin(fma(S, rq[i], L.L0 + pe[i].y), 1.0));
      else t = fma(S, rq[i], (1.0 + L.L0) + pe[i].y);
      acc[i] = fma(p, t, acc[i]);
    } else {      // rq = 1/(den E), as sep_fast_tail_pb with lin(L0, Lc, Ls) = fma(a, T2, L0)
      double in = fma(L.a, b[i].y, lin(L.S0, L.Sc, L.Ss, c[i]));
      in = fma(E[i], fma(L.a, pe[i].y, L.L0), in);
      double t;
      if (REG) t = 1.0 + fmax(-1.0, fmin(rq[i] * in, 1.0));
      else t = fma(rq[i], in, 1.0);
      const double g = pb[i] * (E[i] * rq[i]) * t;
      acc[i] += (OUT && pb[i] <= 0.0) ? 0.0 : g;
    }
  }
}

// Grad fours with the linear delta-f part from the (cell, q, phi) table as well.  Without baryon
// terms (include_baryon = 0: c1 = c3 = 0 and V = 0, so R_SCB = R_SSB = 0 exactly) the lane's
// Sc pc + Ss ps = a mT (SC1 pc + SS1 ps), and T1 = SC1 pc + SS1 ps depends on (cell, y, phi) only,
// so pt[i] = {PD, T1} (one LDS read, as PD alone) and
//   a S = fma(a, fma(mT, T1, Phi), S0')     -- two ops per point instead of three.
// RTA-CE (SEP_CE) in the same launch also takes, per (cell, phi), pe = {TE, T2} with
// TE = -(u^x pc + u^y ps) and T2 = LC pc + LS ps (cell-only lane coefficients, sep_cell_consts):
//   E = E0 + TE,  a (L0 + Lc pc + Ls ps) = fma(a, T2, L0')   -- five ops per point instead of eight.
// SPHI: Phi (b[i].y) is an SGPR operand (F_TS), fma_vvs; BY: the baryon part b T3 (F_BY) joins the linear part
template <int FL, bool REG, bool OUT, bool SPHI = false, bool BY = false>
IS3D_HD void sep_quad_tb_t(const SepLane& L, double mT, const dbl2* b, const dbl2* pt, const dbl2* pe, double* v,
                           double bary = 0.0, const double* t3 = nullptr) {
  constexpr bool needE = FL == SEP_CE;
  double pb[4], q[4], E[4];
#pragma unroll
  for (int i = 0; i < 4; i++) {
    pb[i] = fma(L.D0, b[i].x, L.escw * pt[i].x);
    const double den = fma(L.ssc, b[i].x, L.a);
    E[i] = needE ? L.E0 + pe[i].x : 1.0;
    q[i] = needE ? den * E[i] : den;
  }
  const double q01 = q[0] * q[1], q23 = q[2] * q[3];
  const double r = rcp1(q01 * q23);
  const double r01 = r * q23, r23 = r * q01;
  const double rq[4] = {r01 * q[1], r01 * q[0], r23 * q[3], r23 * q[2]};
#pragma unroll
  for (int i = 0; i < 4; i++) {
    double P = SPHI ? fma_vvs(mT, pt[i].y, b[i].y) : fma(mT, pt[i].y, b[i].y);
    if (BY) P = fma(bary, t3[i], P);
    double in = fma(L.a, P, L.S0);
    if (needE) in = fma(E[i], fma(L.a, pe[i].y, L.L0), in);
    double t;
    if (REG) t = 1.0 + fmax(-1.0, fmin(rq[i] * in, 1.0));
    else t = fma(rq[i], in, 1.0);
    const double g = (needE ? pb[i] * (E[i] * rq[i]) : pb[i] * rq[i]) * t;
    v[i] = (OUT && pb[i] <= 0.0) ? 0.0 : g;
  }
}

// sep_quad_tb_t for a Boltzmann-tail lane (sep_setup allow_tail, L.tail = 1): den == a at every point,
// so with 1/a folded into D0 / escw and the delta-f coefficients unscaled,
//   Grad    acc += pb (1 + S),            S = S0 + mT T1 + Phi                     5 ops per point
//   RTA-CE  acc += pb (1 + L + S / E),    L = L0 + T2, E = E0 + TE, one 1/E per four points
// (pb = w p.dsigma f_eq; regulate clamps delta-f to [-1, 1]; outflow drops points with pb <= 0).
template <int FL, bool REG, bool OUT, bool SPHI = false, bool BY = false>
IS3D_HD void sep_quad_tb_tail_t(const SepLane& L, double mT, const dbl2* b, const dbl2* pt, const dbl2* pe, double* acc,
                                double bary = 0.0, const double* t3 = nullptr) {
  constexpr bool needE = FL == SEP_CE;
  double rE[4] = {0.0, 0.0, 0.0, 0.0};
  if (needE) {
    double E[4];
#pragma unroll
    for (int i = 0; i < 4; i++) E[i] = L.E0 + pe[i].x;
    const double e01 = E[0] * E[1], e23 = E[2] * E[3];
    const double r = rcp1(e01 * e23);
    const double r01 = r * e23, r23 = r * e01;
    rE[0] = r01 * E[1]; rE[1] = r01 * E[0]; rE[2] = r23 * E[3]; rE[3] = r23 * E[2];
  }
#pragma unroll
  for (int i = 0; i < 4; i++) {
    double pb = fma(L.D0, b[i].x, L.escw * pt[i].x);
    if (OUT) pb = (pb <= 0.0) ? 0.0 : pb;
    double P = SPHI ? fma_vvs(mT, pt[i].y, b[i].y) : fma(mT, pt[i].y, b[i].y);
    if (BY) P = fma(bary, t3[i], P);
    double t;
    if (REG) {
      const double S = P + L.S0;
      const double dfv = needE ? fma(S, rE[i], L.L0 + pe[i].y) : S;
      t = 1.0 + fmax(-1.0, fmin(dfv, 1.0));
    } else {   // 1 + S0 and 1 + L0 are lane constants (hoisted by the compiler)
      t = needE ? fma(P + L.S0, rE[i], (1.0 + L.L0) + pe[i].y) : P + (1.0 + L.S0);
    }
    acc[i] = fma(pb, t, acc[i]);
  }
}

// sep_quad_tb_t for a near-tail Grad lane without regulate (sep_setup allow_near, L.near = 1: 1/a folded into
// D0 / escw, delta-f coefficients unscaled, L.ssc = sign 2^-k / a): with u = ssc b' <= e^-kNearX,
// f_eq = (b'/a) / (1 + u) and 1 - sign f_eq = 1 / (1 + u), so a point is
//   pb (1 - u) (1 + (1 - u) S) = pb ((1 + S) - u (1 + 2 S))   (to u^2)          8 ops per point instead of ~11
template <bool OUT, bool SPHI = false, bool BY = false>
IS3D_HD void sep_quad_tb_near_t(const SepLane& L, double mT, const dbl2* b, const dbl2* pt, double* acc,
                                double bary = 0.0, const double* t3 = nullptr) {
#pragma unroll
  for (int i = 0; i < 4; i++) {
    double pb = fma(L.D0, b[i].x, L.escw * pt[i].x);
    if (OUT) pb = (pb <= 0.0) ? 0.0 : pb;
    double P = SPHI ? fma_vvs(mT, pt[i].y, b[i].y) : fma(mT, pt[i].y, b[i].y);
    if (BY) P = fma(bary, t3[i], P);
    const double S1 = P + (1.0 + L.S0);                    // 1 + S
    const double t = fma(-(L.ssc * b[i].x), fma(2.0, S1, -1.0), S1);
    acc[i] = fma(pb, t, acc[i]);
  }
}

// Boltzmann-tail fours with the PD table (pd[i]) and {pc, ps} (c[i], SGPR operands when read by scalar loads)
// instead of the F_TB tables (sep_setup allow_tail: 1/a folded into D0 / escw, delta-f coefficients unscaled):
//   Grad    acc += pb (1 + S),           S = S0 + Sc pc + Ss ps + Phi                  6 ops per point
//   RTA-CE  acc += pb (1 + L + S / E),   L = L0 + Lc pc + Ls ps, E = E0 + Ec pc + Es ps, one 1/E per four
// (pb = w p.dsigma f_eq = fma(D0, b', escw PD); against the fast fours' ~12 (Grad) / ~20 (RTA-CE) ops).
// The F_TB launch's Grad tail lanes in this form read 6 LDS-array cycles per point instead of 8 but were
// 2.2% slower there (IS3D_TAIL_PD, r2d); the per-lane launches (baryon on, RTA-CE with many classes) use it.
template <int FL, bool REG, bool OUT>
IS3D_HD void sep_quad_pd_tail_t(const SepLane& L, const dbl2* c, const dbl2* b, const double* pd, double* acc) {
  constexpr bool needE = FL == SEP_CE;
  double rE[4] = {0.0, 0.0, 0.0, 0.0};
  if (needE) {
    double E[4];
#pragma unroll
    for (int i = 0; i < 4; i++) E[i] = lin(L.E0, L.Ec, L.Es, c[i]);
    const double e01 = E[0] * E[1], e23 = E[2] * E[3];
    const double r = rcp1(e01 * e23);
    const double r01 = r * e23, r23 = r * e01;
    rE[0] = r01 * E[1]; rE[1] = r01 * E[0]; rE[2] = r23 * E[3]; rE[3] = r23 * E[2];
  }
#pragma unroll
  for (int i = 0; i < 4; i++) {
    double pb = fma(L.D0, b[i].x, L.escw * pd[i]);
    if (OUT) pb = (pb <= 0.0) ? 0.0 : pb;
    double t;
    if (REG) {
      const double S = lin(L.S0, L.Sc, L.Ss, c[i]) + b[i].y;
      const double dfv = needE ? fma(S, rE[i], lin(L.L0, L.Lc, L.Ls, c[i])) : S;
      t = 1.0 + fmax(-1.0, fmin(dfv, 1.0));
    } else {   // 1 + S0 and 1 + L0 are lane constants (hoisted by the compiler)
      t = needE ? fma(lin(L.S0, L.Sc, L.Ss, c[i]) + b[i].y, rE[i], lin(1.0 + L.L0, L.Lc, L.Ls, c[i]))
                : lin(L.S0 + 1.0, L.Sc, L.Ss, c[i]) + b[i].y;
    }
    acc[i] = fma(pb, t, acc[i]);
  }
}

IS3D_HD void sep_quad_pd(int flavor,const SepLane& L, const dbl2* c, const dbl2* b, const double* pd, int regulate,
                         int outflow, double* v) {
#define IS3D_QUADPD_CASE(FLV)                                                                     \
  if (flavor == FLV) {                                                                            \
    if (regulate) {                                                                               \
      if (outflow) sep_quad_pd_t<FLV, true, true, true>(L, c, b, pd, v);                              \
      else sep_quad_pd_t<FLV, true, false, true>(L, c, b, pd, v);                                      \
    } else {                                                                                      \
      if (outflow) sep_quad_pd_t<FLV, false, true, true>(L, c, b, pd, v);                              \
      else sep_quad_pd_t<FLV, false, false, true>(L, c, b, pd, v);                                      \
    }                                                                                             \
    return;                                                                                       \
  }
  IS3D_QUADPD_CASE(SEP_GRAD)
  IS3D_QUADPD_CASE(SEP_CE)
  IS3D_QUADPD_CASE(SEP_PTB)
  IS3D_QUADPD_CASE(SEP_FEQ)
#undef IS3D_QUADPD_CASE
}

IS3D_HD void sep_quad(int flavor, const SepLane& L, const dbl2* c, const dbl2* b, int regulate, int outflow, double* v) {
#define IS3D_QUAD_CASE(FLV)                                                                       \
  if (flavor == FLV) {                                                                            \
    if (regulate) {                                                                               \
      if (outflow) sep_quad_t<FLV, true, true>(L, c, b, v);                                       \
      else sep_quad_t<FLV, true, false>(L, c, b, v);                                              \
    } else {                                                                                      \
      if (outflow) sep_quad_t<FLV, false, true>(L, c, b, v);                                      \
      else sep_quad_t<FLV, false, false>(L, c, b, v);                                             \
    }                                                                                             \
    return;                                                                                       \
  }
  IS3D_QUAD_CASE(SEP_GRAD)
  IS3D_QUAD_CASE(SEP_CE)
  IS3D_QUAD_CASE(SEP_PTB)
  IS3D_QUAD_CASE(SEP_FEQ)
#undef IS3D_QUAD_CASE
}

IS3D_HD double sep_point(int flavor, const SepLane& L, dbl2 cs, dbl2 bp, int regulate, int outflow) {
#define IS3D_SEP_CASE(FLV)                                                                               \
  if (flavor == FLV) {                                                                                   \
    if (L.fast) {                                                                                        \
      if (regulate) return outflow ? sep_point_t<FLV, true, true, true>(L, cs, bp)                       \
                                   : sep_point_t<FLV, true, false, true>(L, cs, bp);                     \
      return outflow ? sep_point_t<FLV, false, true, true>(L, cs, bp)                                    \
                     : sep_point_t<FLV, false, false, true>(L, cs, bp);                                  \
    }                                                                                                    \
    if (regulate) return outflow ? sep_point_t<FLV, true, true, false>(L, cs, bp)                        \
                                 : sep_point_t<FLV, true, false, false>(L, cs, bp);                      \
    return outflow ? sep_point_t<FLV, false, true, false>(L, cs, bp)                                     \
                   : sep_point_t<FLV, false, false, false>(L, cs, bp);                                   \
  }
  IS3D_SEP_CASE(SEP_GRAD)
  IS3D_SEP_CASE(SEP_CE)
  IS3D_SEP_CASE(SEP_PTB)
  IS3D_SEP_CASE(SEP_FEQ)
#undef IS3D_SEP_CASE
  return 0.0;
}

// sqrt(v) for normal v > 0: v_rsq_f64 (5e-8) + one Newton-Goldschmidt step (~4e-15 relative);
// IEEE sqrt on the host
IS3D_HD double sqrt_nr(double v) {
#if defined(__HIP_DEVICE_COMPILE__)
  const double y = __builtin_amdgcn_rsq(v);
  const double g = v * y, h = 0.5 * y;
  return fma(g, fma(-g, h, 0.5), g);
#else
  return sqrt(v);
#endif
}

// Modified (PTM/PTB/PTMA) lane: p_mod = mT (ch Uc + sh Us) + (pc Vc + ps Vs)  (MomentumSpectra.cpp:932-982
// without the iterative refinement, which only changes rounding: A is linear).  Writing
// p_mod = mT U + W with U = ch Uc + sh Us per (cell, y) and W = pc Vc + ps Vs per (cell, phi),
//   E_mod^2 = m^2 + mT^2 |U|^2 + 2 mT (U.Vc) pc + 2 mT (U.Vs) ps + |W|^2
// so a point needs the lane's linear form E0 + Ec pc + Es ps plus Qv = |W|^2 from the per-(cell, phi)
// LDS table (modqv) instead of rebuilding the 3-vector (E_mod^2 >= m^2 >= 0.019 GeV^2 for every
// hadron, so the expanded form loses nothing measurable to cancellation).
// f = |renorm| / (exp(E_mod/T_mod - chem) + sign) is evaluated as |renorm| en / (1 + sign en) with
// en = exp(chem - E_mod/T_mod): u.p > 0 bounds en by e^chem and, for bosons (no baryon number),
// below 1, so 1 + sign en lies in ~[1e-3, 2] and two points can share one reciprocal; en -> 0
// where the reference's exp overflows to 1/inf = 0.  |renorm| is folded into p.dsigma.
// Exp-table units: the record's directions are scaled by sig = (1/T_mod) kModTabN/ln2
// (mod_scale_record), so E0 + Qv + ... = (sig E_mod)^2 and sqrt of it is exp_tab's argument; on the
// table lanes (!clamp) e^chem is folded out of the exponential into sign and the p.dsigma
// coefficients (en = e^chem e^-E/T: en / (1 + sign en) = e^chem e / (1 + (sign e^chem) e)), so a point
// evaluates e^(-sig E_mod) alone.
// Plus form (IS3D_MOD_PLUS, table lanes): f = 1 / (e^x + sign e^chem) e^chem with x = E_mod / T_mod evaluated as
//   f = 2^-k / (E + s),  E = e^x 2^-k,  s = sign e^chem 2^-k,  2^-k e^chem folded into the p.dsigma coefficients,
// where k = floor(x_min / ln2) over the lane's phi points (from mod_setup's lower bound) keeps E in [~1, 2^250]:
// four denominators multiply without overflow and the scale costs nothing per point (2^-k enters the range
// reduction's shift constant, shiftk = 1.5 2^52 - N k).  The numerator is 1, so a point saves the en x q_j product
// of the en form (f = en / (1 + s en)); it is also the reference's own form, 1 / (exp(E/T - chem) + sign)
// (MomentumSpectra.cpp:980).  Lanes whose phi range exceeds 250 binades take the clamped en form.
#ifndef IS3D_MOD_PLUS
#define IS3D_MOD_PLUS 1
#endif
// Boltzmann-tail lanes (IS3D_MOD_TAIL): where |s| < 2^-55 <= 2^-55 E at every point, E + s == E exactly, so
// f = 2^-k / E = e^-(x - k ln2) 2^-k: the point evaluates that exponential directly (the shift constant
// 1.5 2^52 + N k) and skips the denominators and the shared reciprocal (mod_quad_tab_tail_t).  Decided once
// per wavefront (mod_setup allow_tail): a wave whose lanes straddle the bound runs the normal fours only
#ifndef IS3D_MOD_TAIL
#define IS3D_MOD_TAIL 1
#endif
#ifndef IS3D_MOD_WIDE_TAIL
#define IS3D_MOD_WIDE_TAIL 1
#endif
#ifndef IS3D_MOD_EXACT
#define IS3D_MOD_EXACT 1
#endif
struct ModExpCoef { double a[kModExpDeg]; };

struct ModLane {
  double E0, Ec, Es, D0, Dc, Ds, chemm, sign;   // table lanes: sign = sign e^chem, D = |renorm| e^chem D
                                                // (plus form: both x 2^-k)
  double mT, Dw;               // table form (mod_quad_tab_t): E_mod^2 = E0 + Qv + mT T2, p.dsigma = D0 + Dw PDm
  double shiftk;               // plus form: 1.5 2^52 - kModTabN k (the lane's 2^-k in the range reduction)
  ModExpCoef et;               // pinned once per lane setup, reused by every phi point
  const double* etab;          // 2^(j/kModTabN) table (LDS on the device)
  int skip, clamp;   // clamp: some point's exp argument may leave the table lanes' domain (exp_clamped instead)
  int tail;          // IS3D_MOD_TAIL: Boltzmann-tail table lane (shiftk = 1.5 2^52 + N k, mod_quad_tab_tail_t)
};

// Qv = |pc Vc + ps Vs|^2 for one (cell, phi), exp-table units (sig^2)
IS3D_HD double modqv(const double* R, dbl2 cs) {
  const double wx = fma(cs.x, R[R_VCX], cs.y * R[R_VSX]);
  const double wy = fma(cs.x, R[R_VCY], cs.y * R[R_VSY]);
  const double wz = fma(cs.x, R[R_VCZ], cs.y * R[R_VSZ]);
  return fma(wx, wx, fma(wy, wy, wz * wz));
}

// ln2 / kModTabN: sig E_mod x this = E_mod / T_mod
static constexpr double kLn2overN = 1.0 / kModInvLn2xN;
// table lanes: E_mod / T_mod below 1e6 (exp_tab's integer part fits the low word; beyond e^-745 en is
// 0 anyway) and |chem| < 30: where e^(-E/T) underflows (E/T > 745) the reference's exp(E/T - chem)
// overflows too (E/T - chem > 715), so folding e^chem out loses nothing, and four 1 + sign e^chem e
// factors multiply without overflow in the quad reciprocal
static constexpr double kModTabX = 1.0e6, kModTabChem = 30.0;
#ifndef IS3D_MODQ_ACC
#define IS3D_MODQ_ACC 1
#endif
#ifndef IS3D_MOD_SQ_BOUNDS
#define IS3D_MOD_SQ_BOUNDS 1
#endif

// e^x for xN = x kModTabN/ln2 with the modified lanes' table and polynomial (mod_setup's e^chem)
IS3D_HD double mod_exp(const double* etab, double xN) {
  if (IS3D_MOD_TAB_BITS == IS3D_EXP_TAB_BITS) return exp_tab(exp_tab_coef(), etab, xN);   // the shared table
  const double sh = 6755399441055744.0;
  const double t = xN + sh;
  const double rs = xN - (t - sh);
  const int ki = (int)(unsigned)__builtin_bit_cast(unsigned long long, t);
  double p = kModExpA[kModExpDeg - 1];
#pragma unroll
  for (int i = kModExpDeg - 2; i >= 0; i--) p = fma(p, rs, kModExpA[i]);
  const double T = etab[ki & (kModTabN - 1)];
  return ldexp(fma(T, rs * p, T), ki >> IS3D_MOD_TAB_BITS);
}

// mod_setup's skip test alone (same operations, IS3D_MOD_SQ_BOUNDS form), for an early branch past the setup
IS3D_HD bool mod_skips(const double* R, const double* Y, double mT, double m2, double pT, double baryon, bool ymu = true) {
  const double ux = Y[Y_MUX], uy = Y[Y_MUY], uz = Y[Y_MUZ];
  const double u2 = ymu ? Y[Y_MU2] : fma(ux, ux, fma(uy, uy, uz * uz));
  const double sig = R[R_INVTM] * kModInvLn2xN, m2s = m2 * (sig * sig);
  const double mu = mT * (ymu ? Y[Y_MU] : sqrt(u2));
  const double lo = mu - pT * R[R_VB];
  const double thr = (kExpMax + 1.0 + baryon * R[R_CHEMM]) * kModInvLn2xN;
  return thr < 0.0 || (lo > 0.0 && (m2s + lo * lo) * (1.0 - 2e-12) > thr * thr);
}

// KJX > 0 (k_spectra's table lanes; -1: nx points, the host emulator): MW / MT are the lane's {PDm, Qv} and T2 rows of KJX points.  A lane whose bounds
// span more than 250 binades (wide) takes its exact smallest / largest X over those points instead (IS3D_MOD_EXACT): the
// bounds |mT U| -+ pT |V|max are loose where pT |V| is large, and a lane found wide by them went to the clamped en form
// (1.6x the normal fours' instructions) although its points spanned a median 134 binades (config 2 PTM, host census)
template <int KJX = 0>
IS3D_HD void mod_setup(const double* R, const double* Y, double mT, double m2, double pT, double sign, double baryon,
                       double renorm_abs, const double* etab, ModLane& L, bool ymu = true, bool allow_tail = false,
                       const dbl2* MW = nullptr, const double* MT = nullptr, int nx = KJX) {
  const double ux = Y[Y_MUX], uy = Y[Y_MUY], uz = Y[Y_MUZ];   // sig U
  const double u2 = ymu ? Y[Y_MU2] : fma(ux, ux, fma(uy, uy, uz * uz));
  const double sig = R[R_INVTM] * kModInvLn2xN, m2s = m2 * (sig * sig);
  L.E0 = fma(mT * mT, u2, m2s);
  const double tm = 2.0 * mT;
  L.Ec = tm * fma(ux, R[R_VCX], fma(uy, R[R_VCY], uz * R[R_VCZ]));
  L.Es = tm * fma(ux, R[R_VSX], fma(uy, R[R_VSY], uz * R[R_VSZ]));
  L.mT = mT;
  L.chemm = baryon * R[R_CHEMM];
  for (int i = 0; i < kModExpDeg; i++) L.et.a[i] = kconst(kModExpA[i]);
  L.etab = etab;
  // | |mT U| - pT |V|max | <= |p_mod| <= |mT U| + pT |V|max (sig units): if even the smallest E_mod
  // overflows exp, every phi point is exactly 0; if the largest could leave the table lanes' domain
  // the lane takes the clamped exp
  const double mu = mT * (ymu ? Y[Y_MU] : sqrt(u2));
  const double lo = mu - pT * R[R_VB], hi = mu + pT * R[R_VB];
#if IS3D_MOD_SQ_BOUNDS
  // the same two tests on squares (no sqrt): skip when sig E_min (1 - 1e-12) exceeds
  // thr = (kExpMax + 1 + chem) N/ln2 -- always when thr < 0, as E_min >= 0
  const double thr = (kExpMax + 1.0 + L.chemm) * kModInvLn2xN, xm = kModTabX * kModInvLn2xN;
  L.skip = (thr < 0.0 || (lo > 0.0 && (m2s + lo * lo) * (1.0 - 2e-12) > thr * thr)) ? 1 : 0;
  L.clamp = ((m2s + hi * hi) < xm * xm && fabs(L.chemm) < kModTabChem) ? 0 : 1;
#else
  const double emin = (lo > 0.0) ? sqrt(m2s + lo * lo) * (1.0 - 1e-12) : 0.0;
  L.skip = (emin * kLn2overN - L.chemm > kExpMax + 1.0) ? 1 : 0;
  const double emax = sqrt(m2s + hi * hi) * kLn2overN;
  L.clamp = (emax < kModTabX && fabs(L.chemm) < kModTabChem) ? 0 : 1;
#endif
  int k = 0, wide = 0;
#if IS3D_MOD_PLUS
  if (!L.clamp) {
    // k = floor(x_min / ln2) from the lane's smallest sig E_mod (a lower bound of it: rounding down only
    // raises E by a factor < 2); the normal fours need the largest point within 250 binades of 2^k (wide: not)
    double e2 = m2s + (lo > 0.0 ? lo * lo : 0.0), e2h = m2s + hi * hi;
    auto scale = [&]() {
#if defined(__HIP_DEVICE_COMPILE__)
      const double emin = e2 * __builtin_amdgcn_rsq(e2);
#else
      const double emin = sqrt(e2);
#endif
      k = (int)(emin * ((1.0 - 1e-6) / kModTabN));
      const double xk = (k + 250.0) * kModTabN;
      wide = (e2h < xk * xk) ? 0 : 1;
    };
    scale();
    if constexpr (KJX != 0) {   // KJX = -1: nx points (the host emulator)
      if (IS3D_MOD_EXACT && MW) {
        // the exact range of the lane's points (the loops' own X expression); a wave-uniform branch on the device
#if defined(__HIP_DEVICE_COMPILE__)
        int aw = __any(wide);
        asm volatile("" : "+v"(aw));
        if (aw) {
#else
        {
#endif
          if (wide) {
            double mn = 1.0e300, mx = 0.0;
#pragma unroll 8
            for (int j = 0; j < (KJX > 0 ? KJX : nx); j++) {
              const double X = fma(mT, MT[j], L.E0 + MW[j].y);
              mn = fmin(mn, X); mx = fmax(mx, X);
            }
            e2 = mn; e2h = mx;
            scale();
          }
        }
      }
    }
  }
#endif
  // only callers that evaluate tail lanes with mod_quad_tab_tail_t pass allow_tail.  The tail form has no
  // denominators (no product of four), so a wide lane is a tail lane too when its sign term is negligible
  // (IS3D_MOD_WIDE_TAIL; before, every wide lane took the clamped en form: 5% of config 2's PTM wavefronts, at 1.6x the
  // normal fours' instructions)
  L.tail = (IS3D_MOD_PLUS && IS3D_MOD_TAIL && allow_tail && !L.clamp && (IS3D_MOD_WIDE_TAIL || !wide) &&
            L.chemm * 1.4426950408889634 < k - 55) ? 1 : 0;
#if defined(__HIP_DEVICE_COMPILE__)
  if (IS3D_MOD_TAIL && allow_tail) {   // one decision per wavefront, passed through a VGPR (see sep_setup)
    int t = __all(L.tail);
    asm volatile("" : "+v"(t));
    L.tail = t;
  }
#endif
  if (wide && !L.tail) L.clamp = 1;
  // e^chem of the table lanes (1 for mesons and without baryon chemistry: a wave-uniform skip there)
  double ec = 1.0;
  if (!L.clamp && L.chemm != 0.0) ec = mod_exp(etab, L.chemm * kModInvLn2xN);
  if (L.clamp) k = 0;
  L.shiftk = 6755399441055744.0 + (L.tail ? 1.0 : -1.0) * ((double)k * kModTabN);
  const double d = ldexp(renorm_abs * ec, -k);
  L.sign = ldexp(sign * ec, -k);
  L.D0 = d * (mT * Y[Y_MD]); L.Dc = d * Y[Y_WDX]; L.Ds = d * Y[Y_WDY];
  L.Dw = d * Y[Y_W];
}

// The Fermi/Bose factor of one point as num / q: clamped lanes num = en = e^(chem - E_mod/T_mod),
// q = 1 + sign en; table lanes in the plus form num = 1, q = E + s (see ModLane), in the en form (IS3D_MOD_PLUS 0)
// num = en = e^(-E_mod/T_mod), q = 1 + s en.  X = (sig E_mod)^2: one Newton step of the v_rsq_f64 estimate y
// folded into the exp argument, sig E_mod = g v with g = X y, v = 1.5 - 0.5 g y, and the range reduction folded
// into the product (t = fma(g, v, shift) rounds g v to the integer K exactly, rs = fma(g, v, shift - t))
// rsq estimate of the table lanes' X = (sig E_mod)^2 (v_rsq_f64, 16 cycles per wave on MI355X, tools/microbench.hip; v_rsq_f32
// with the two conversions costs the same 16.5 and measured no faster, profiles/round5_r5a_ab_mod.log)
IS3D_HD double mod_rsq(double X) {
#if defined(__HIP_DEVICE_COMPILE__)
  return __builtin_amdgcn_rsq(X);
#else
  return 1.0 / sqrt(X);
#endif
}

template <bool CLAMP>
IS3D_HD void mod_nq_x(const ModLane& L, double X, double& num, double& q) {
  if (CLAMP) {
    num = exp_clamped(exp_coef(), fma(-sqrt_nr(X), kLn2overN, L.chemm));
    q = fma(L.sign, num, 1.0);
    return;
  }
  const double y = mod_rsq(X);
  const double g = IS3D_MOD_PLUS ? X * y : -(X * y);
  const double v = fma(-0.5, X * y * y, 1.5);
  const double sh = IS3D_MOD_PLUS ? L.shiftk : kconst(6755399441055744.0);
  const double t = fma(g, v, sh);
  const double rs = fma(g, v, sh - t);
  const int ki = (int)(unsigned)__builtin_bit_cast(unsigned long long, t);
  double p = L.et.a[kModExpDeg - 1];
#pragma unroll
  for (int i = kModExpDeg - 2; i >= 0; i--) p = fma(p, rs, L.et.a[i]);
  const double T = L.etab[ki & (kModTabN - 1)];
  const double e = ldexp(fma(T, rs * p, T), ki >> IS3D_MOD_TAB_BITS);
  if (IS3D_MOD_PLUS) { num = 1.0; q = e + L.sign; }
  else { num = e; q = fma(L.sign, e, 1.0); }
}

// the same from the lane's linear form (qv = modqv of the cell at this phi)
template <bool CLAMP>
IS3D_HD void mod_nq(const ModLane& L, dbl2 cs, double qv, double& num, double& q) {
  mod_nq_x<CLAMP>(L, fma(L.Ec, cs.x, fma(L.Es, cs.y, L.E0 + qv)), num, q);
}

template <bool OUT, bool CLAMP>
IS3D_HD double mod_point_t(const ModLane& L, dbl2 cs, double qv) {
  double num, q;
  mod_nq<CLAMP>(L, cs, qv, num, q);
  const double pds = lin(L.D0, L.Dc, L.Ds, cs);
  const double r = pds * (num * rcp1(q));
  return (OUT && pds <= 0.0) ? 0.0 : r;
}

// two points, one reciprocal: f_0 = num_0 q_1 / (q_0 q_1)
IS3D_HD void mod_pair_f(double n0, double q0, double n1, double q1, double& f0, double& f1) {
  const double r = rcp1(q0 * q1);
  f0 = n0 * (r * q1);
  f1 = n1 * (r * q0);
}

template <bool OUT, bool CLAMP>
IS3D_HD void mod_pair_t(const ModLane& L, dbl2 c0, dbl2 c1, dbl2 qv, double& v0, double& v1) {
  double n0, q0, n1, q1, f0, f1;
  mod_nq<CLAMP>(L, c0, qv.x, n0, q0);
  mod_nq<CLAMP>(L, c1, qv.y, n1, q1);
  mod_pair_f(n0, q0, n1, q1, f0, f1);
  const double pds0 = lin(L.D0, L.Dc, L.Ds, c0), pds1 = lin(L.D0, L.Dc, L.Ds, c1);
  v0 = (OUT && pds0 <= 0.0) ? 0.0 : pds0 * f0;
  v1 = (OUT && pds1 <= 0.0) ? 0.0 : pds1 * f1;
}

// four points, one reciprocal (the four denominators lie in ~[1e-3, 2] (en form) or [~1, 2^250] (plus form),
// so their product is normal): rq_i = 1 / q_i as r q_j q_k q_l
IS3D_HD void mod_quad_rq(const double* q, double* rq) {
  const double q01 = q[0] * q[1], q23 = q[2] * q[3];
  const double r = rcp1(q01 * q23);
  const double r01 = r * q23, r23 = r * q01;
  rq[0] = r01 * q[1]; rq[1] = r01 * q[0]; rq[2] = r23 * q[3]; rq[3] = r23 * q[2];
}

template <bool OUT, bool CLAMP>
IS3D_HD void mod_quad_t(const ModLane& L, const dbl2* c, dbl2 qa, dbl2 qb, double* v) {
  double num[4], q[4], rq[4];
  const double qv[4] = {qa.x, qa.y, qb.x, qb.y};
#pragma unroll
  for (int i = 0; i < 4; i++) mod_nq<CLAMP>(L, c[i], qv[i], num[i], q[i]);
  mod_quad_rq(q, rq);
#pragma unroll
  for (int i = 0; i < 4; i++) {
    const double pds = lin(L.D0, L.Dc, L.Ds, c[i]);
    const double g = pds * (num[i] * rq[i]);
    v[i] = (OUT && pds <= 0.0) ? 0.0 : g;
  }
}

// ---- table form of the modified path (k_spectra).  Per (cell, phi) the workgroup stores
//   MW = {PDm, Qv},  PDm = dsigma_x pc + dsigma_y ps,  Qv = |W|^2  (W = pc Vc + ps Vs)
// and per (cell, q, phi)  T2 = 2 U_q . W  (modt2), so a point needs
//   E_mod^2 = fma(mT, T2, E0 + Qv)   and   p.dsigma |renorm| = fma(Dw, PDm, D0)
// -- 3 VALU ops where the lane's linear forms took 5 -- and no {pc, ps} operands.
IS3D_HD double modpdm(const double* R, dbl2 cs) { return fma(R[R_DAX], cs.x, R[R_DAY] * cs.y); }
IS3D_HD double modt2(const double* R, const double* Y, dbl2 cs) {
  const double wx = fma(cs.x, R[R_VCX], cs.y * R[R_VSX]);
  const double wy = fma(cs.x, R[R_VCY], cs.y * R[R_VSY]);
  const double wz = fma(cs.x, R[R_VCZ], cs.y * R[R_VSZ]);
  return 2.0 * fma(Y[Y_MUX], wx, fma(Y[Y_MUY], wy, Y[Y_MUZ] * wz));
}

// mod_nq_x for four points in stages: the four range reductions, then the four table reads issued
// together, then the four polynomials (independent of the reads), then the products -- so one LDS
// latency is waited for per four points instead of per one or two (same operations, same results)
#ifndef IS3D_MOD_STAGED
#define IS3D_MOD_STAGED 1
#endif
#ifndef IS3D_MOD_IEXP
#define IS3D_MOD_IEXP 0
#endif
// m 2^k for a normal m and a k that keeps the result normal: k added to the exponent field of the high word
IS3D_HD double exp_field_add(double m, int k) {
  const unsigned long long b = __builtin_bit_cast(unsigned long long, m);
  const unsigned hi = (unsigned)(b >> 32) + ((unsigned)k << 20), lo = (unsigned)b;
  return __builtin_bit_cast(double, ((unsigned long long)hi << 32) | lo);
}
template <bool CLAMP, bool TAIL = false>
IS3D_HD void mod_nq4(const ModLane& L, const double* X, double* num, double* q) {
  if (!TAIL && (CLAMP || !IS3D_MOD_STAGED)) {
#pragma unroll
    for (int i = 0; i < 4; i++) mod_nq_x<CLAMP>(L, X[i], num[i], q[i]);
    return;
  }
  double t[4], rs[4], T[4], p[4];
  int ki[4];
  const double sh = IS3D_MOD_PLUS ? L.shiftk : kconst(6755399441055744.0);
#pragma unroll
  for (int i = 0; i < 4; i++) {
    const double y = mod_rsq(X[i]);
    const double g = (IS3D_MOD_PLUS && !TAIL) ? X[i] * y : -(X[i] * y);
    const double v = fma(-0.5, X[i] * y * y, 1.5);
    t[i] = fma(g, v, sh);
    rs[i] = fma(g, v, sh - t[i]);
    ki[i] = (int)(unsigned)__builtin_bit_cast(unsigned long long, t[i]);
  }
#pragma unroll
  for (int i = 0; i < 4; i++) T[i] = L.etab[ki[i] & (kModTabN - 1)];
#pragma unroll
  for (int i = 0; i < 4; i++) {
    double a = L.et.a[kModExpDeg - 1];
#pragma unroll
    for (int k = kModExpDeg - 2; k >= 0; k--) a = fma(a, rs[i], L.et.a[k]);
    p[i] = rs[i] * a;
  }
#pragma unroll
  for (int i = 0; i < 4; i++) {
    const double m = fma(T[i], p[i], T[i]);
    // plus-form normal lanes: E = m 2^K lies in [~1/2, 2^251] (mod_setup's k), so the scale can go straight into
    // the exponent field (one INT32 shift-add on the high word instead of v_ldexp_f64: IS3D_MOD_IEXP); the tail
    // and en forms can underflow and keep ldexp
    const double e = (IS3D_MOD_IEXP && IS3D_MOD_PLUS && !TAIL) ? exp_field_add(m, ki[i] >> IS3D_MOD_TAB_BITS)
                                                                : ldexp(m, ki[i] >> IS3D_MOD_TAB_BITS);
    if (TAIL) { num[i] = e; q[i] = 1.0; }
    else if (IS3D_MOD_PLUS) { num[i] = 1.0; q[i] = e + L.sign; }
    else { num[i] = e; q[i] = fma(L.sign, e, 1.0); }
  }
}

// four points, one reciprocal, accumulated into acc: f_i = num_i / q_i = num_i q_j (1 / q_i q_j) with j the
// pair partner, so acc_i = fma(pds_i num_i q_j, r_ij, acc_i) (plus form: num_i = 1) -- 4 ops per point after the
// shared reciprocal
template <bool OUT, bool CLAMP, typename ACC>
IS3D_HD void mod_quad_tab_t(const ModLane& L, const dbl2* mw, const double* mt, ACC acc) {
  double num[4], q[4], X[4];
#pragma unroll
  for (int i = 0; i < 4; i++) X[i] = fma(L.mT, mt[i], L.E0 + mw[i].y);
  mod_nq4<CLAMP>(L, X, num, q);
  const double q01 = q[0] * q[1], q23 = q[2] * q[3];
  const double r = rcp1(q01 * q23);
  const double rp[4] = {r * q23, r * q23, r * q01, r * q01};
  const double h[4] = {num[0] * q[1], num[1] * q[0], num[2] * q[3], num[3] * q[2]};
#pragma unroll
  for (int i = 0; i < 4; i++) {
    double pds = fma(L.Dw, mw[i].x, L.D0);
    if (OUT) pds = (pds <= 0.0) ? 0.0 : pds;
    acc[i] = fma(pds * h[i], rp[i], acc[i]);
  }
}

// Boltzmann-tail table lane: f 2^k = e^-(x - k ln2) per point, no denominators
template <bool OUT, typename ACC>
IS3D_HD void mod_quad_tab_tail_t(const ModLane& L, const dbl2* mw, const double* mt, ACC acc) {
  double num[4], q[4], X[4];
#pragma unroll
  for (int i = 0; i < 4; i++) X[i] = fma(L.mT, mt[i], L.E0 + mw[i].y);
  mod_nq4<false, true>(L, X, num, q);
#pragma unroll
  for (int i = 0; i < 4; i++) {
    double pds = fma(L.Dw, mw[i].x, L.D0);
    if (OUT) pds = (pds <= 0.0) ? 0.0 : pds;
    acc[i] = fma(pds, num[i], acc[i]);
  }
}

template <bool OUT, bool CLAMP>
IS3D_HD void mod_pair_tab_t(const ModLane& L, dbl2 mw0, dbl2 mw1, double mt0, double mt1, double& v0, double& v1) {
  double n0, q0, n1, q1, f0, f1;
  mod_nq_x<CLAMP>(L, fma(L.mT, mt0, L.E0 + mw0.y), n0, q0);
  mod_nq_x<CLAMP>(L, fma(L.mT, mt1, L.E0 + mw1.y), n1, q1);
  mod_pair_f(n0, q0, n1, q1, f0, f1);
  const double pds0 = fma(L.Dw, mw0.x, L.D0), pds1 = fma(L.Dw, mw1.x, L.D0);
  v0 = (OUT && pds0 <= 0.0) ? 0.0 : pds0 * f0;
  v1 = (OUT && pds1 <= 0.0) ? 0.0 : pds1 * f1;
}

// two points of a modified lane from its linear forms and Qv (no q-row table)
template <bool OUT, bool CLAMP>
IS3D_HD void mod_pair_lane_t(const ModLane& L, dbl2 c0, dbl2 c1, double qv0, double qv1, double& v0, double& v1) {
  double n0, q0, n1, q1, f0, f1;
  mod_nq<CLAMP>(L, c0, qv0, n0, q0);
  mod_nq<CLAMP>(L, c1, qv1, n1, q1);
  mod_pair_f(n0, q0, n1, q1, f0, f1);
  const double pds0 = lin(L.D0, L.Dc, L.Ds, c0), pds1 = lin(L.D0, L.Dc, L.Ds, c1);
  v0 = (OUT && pds0 <= 0.0) ? 0.0 : pds0 * f0;
  v1 = (OUT && pds1 <= 0.0) ? 0.0 : pds1 * f1;
}

IS3D_HD void mod_quad(const ModLane& L, const dbl2* c, dbl2 qa, dbl2 qb, int outflow, double* v) {
  if (L.clamp) {
    if (outflow) mod_quad_t<true, true>(L, c, qa, qb, v);
    else mod_quad_t<false, true>(L, c, qa, qb, v);
  } else {
    if (outflow) mod_quad_t<true, false>(L, c, qa, qb, v);
    else mod_quad_t<false, false>(L, c, qa, qb, v);
  }
}

IS3D_HD double mod_point(const ModLane& L, dbl2 cs, double qv, int outflow) {
  if (L.clamp) return outflow ? mod_point_t<true, true>(L, cs, qv) : mod_point_t<false, true>(L, cs, qv);
  return outflow ? mod_point_t<true, false>(L, cs, qv) : mod_point_t<false, false>(L, cs, qv);
}

IS3D_HD void mod_pair(const ModLane& L, dbl2 c0, dbl2 c1, dbl2 qv, int outflow, double& v0, double& v1) {
  if (L.clamp) {
    if (outflow) mod_pair_t<true, true>(L, c0, c1, qv, v0, v1);
    else mod_pair_t<false, true>(L, c0, c1, qv, v0, v1);
  } else {
    if (outflow) mod_pair_t<true, false>(L, c0, c1, qv, v0, v1);
    else mod_pair_t<false, false>(L, c0, c1, qv, v0, v1);
  }
}

}  // namespace is3d

