// rsc_core.h — per-lane numeric core of the MI355X RANSAC pose engine.
//
// Every function here runs in ONE lane for ONE hypothesis (SIMT over hypotheses, see DESIGN.md
// "Kernel mapping").  Small matrices live in VGPRs with compile-time indices (all loops with
// static bounds are unrolled; data-dependent loops are written as unrolled, predicated sweeps so
// that no register array is ever indexed dynamically).  The 12x12 symmetric eigenproblem of EPnP
// lives in a per-lane LDS slab (LaneMat, element-major: element e of lane l at base[e*stride + l],
// so a wave's 64 lanes touch 64 consecutive doubles — conflict-free ds_read_b64/ds_write_b64).
//
// Algorithms follow the reference solvers (src/PnPsolver.cpp, src/Sim3Solver.cpp) and the Eigen
// routines they call (SelfAdjointEigenSolver, JacobiSVD+ColPivHouseholderQR, Matrix3d::inverse,
// Quaternion::toRotationMatrix).  Arithmetic contract: sums left to right in index
// order except the 3-term reductions of fixed-size Eigen expressions, which follow Eigen 3.3 on the
// reference's x86-64 SSE2 build (`ered3`, `emv3d_row` below); no FMA contraction (compiled with
// -ffp-contract=off), IEEE-correct division and sqrt.
//
// The header is also compiled for the host by the test-only emulation library
// (tests/hostemu/), so the device arithmetic can be checked against the oracle on a CPU.
#pragma once
#include <cstdint>
#include <cfloat>
#include <cmath>
#include <utility>

#if defined(__HIPCC__)
#include <hip/hip_runtime.h>
#define RSC_HD __host__ __device__ __forceinline__
#else
#define RSC_HD inline
#endif
#define RSC_UNROLL _Pragma("unroll")
// End of a data-dependent loop body whose last statement is conditional: a convergent no-op that
// keeps LLVM from tail-duplicating the latch.  Without it the loop gets two backedges and
// LoopSimplify splits it into a nested loop, in which the lanes of a wave that took different
// backedges wait for each other (measured 2.6x on the 12x12 eigensolver).
#if defined(__HIP_DEVICE_COMPILE__)
#define RSC_LOOP_FENCE() __builtin_amdgcn_wave_barrier()
#else
#define RSC_LOOP_FENCE() ((void)0)
#endif
// A scheduling fence (no instruction): the scheduler keeps every instruction on its side, so a
// straight-line sequence of independent blocks does not have all their loads hoisted to the top
// (the register live ranges stay one block long).
#if defined(__HIP_DEVICE_COMPILE__)
#define RSC_SCHED_FENCE() __builtin_amdgcn_sched_barrier(0)
#else
#define RSC_SCHED_FENCE() ((void)0)
#endif

namespace rsc {

// Bounded poll of a hand-off flag (the split eigen stage's pub / ack words): v = load() until pred(v)
// holds, pause() between polls, at most `limit` polls.  Returns false when it gave up — the caller
// then raises the launch's fault word, so a lost hand-off is an error status, never a silently
// wrong eigenvector.  Compiled for the host too (tests/hostemu: the give-up path at limit 1).
template <class Load, class Pause, class Pred>
RSC_HD bool poll_until(int limit, Load load, Pause pause, Pred pred, int& v) {
    for (int it = 0; it < limit; ++it) {
        v = load();
        if (pred(v)) return true;
        pause();
    }
    return false;
}

template <typename S> struct lim;
template <> struct lim<double> {
    RSC_HD static double eps() { return 2.220446049250313080847e-16; }
    RSC_HD static double min() { return 2.2250738585072013830903e-308; }
};
template <> struct lim<float> {
    RSC_HD static float eps() { return 1.1920928955078125e-07f; }
    RSC_HD static float min() { return 1.17549435082228750797e-38f; }
};

RSC_HD double rsqrt_(double x) { return sqrt(x); }

// 3-term reduction of a fixed-size Eigen expression that cannot use SIMD packets — a coefficient of
// a product / dot / squared norm over a row of a column-major matrix, or any float 3-vector (3 < 4
// lanes): Eigen's redux_novec_unroller halves the index range, a0 + (a1 + a2).
template <typename S> RSC_HD S ered3(S a0, S a1, S a2) { return a0 + (a1 + a2); }
// Row r of a Matrix3d * Vector3d assigned to a Vector3d: rows 0-1 are one Packet2d multiply-add
// chain in index order, row 2 is the coefficient path.
template <typename S> RSC_HD S emv3d_row(int r, S a0, S a1, S a2) { return r < 2 ? (a0 + a1) + a2 : ered3(a0, a1, a2); }

// sqrt(x) for x in [1, 4) and 1/u for |u| in [1, 2), correctly rounded, with shorter chains (device).
// The compiler's IEEE expansions add range handling around the core: sqrt scales x below 2^-767
// (v_cmp -> s_cselect -> v_ldexp, a VALU-SALU-VALU round trip) and fixes up +-0 / inf after it;
// 1/u pre-scales with v_div_scale and post-fixes with v_div_fixup.  In these ranges every one of
// those steps returns its input (and v_div_fmas is a plain fma), so the core instructions issued
// directly give the same bits with 3-4 fewer dependent steps each: make_givens' 1 + t^2 in [1, 2]
// and sqrt(1 + t^2) in [1, sqrt 2] are exactly these cases.  tests/test_gpu_math.py checks both
// against IEEE numpy over their ranges.
RSC_HD double sqrt_unit(double x) {
#if defined(__HIP_DEVICE_COMPILE__)
    const double y = __builtin_amdgcn_rsq(x);
    double g = x * y, h = y * 0.5;
    const double r = __builtin_fma(-h, g, 0.5);
    g = __builtin_fma(g, r, g);
    h = __builtin_fma(h, r, h);
    double d = __builtin_fma(-g, g, x);
    g = __builtin_fma(d, h, g);
    d = __builtin_fma(-g, g, x);
    return __builtin_fma(d, h, g);
#else
    return sqrt(x);
#endif
}
RSC_HD double recip_unit(double u) {
#if defined(__HIP_DEVICE_COMPILE__)
    double r = __builtin_amdgcn_rcp(u);
    double e = __builtin_fma(-u, r, 1.0);
    r = __builtin_fma(r, e, r);
    e = __builtin_fma(-u, r, 1.0);
    r = __builtin_fma(r, e, r);
    e = __builtin_fma(-u, r, 1.0);  // q = 1 * r = r: the expansion's residual and correction
    return __builtin_fma(e, r, r);
#else
    return 1.0 / u;
#endif
}
RSC_HD float sqrt_unit(float x) { return sqrtf(x); }
RSC_HD float recip_unit(float u) { return 1.0f / u; }
RSC_HD float rsqrt_(float x) { return sqrtf(x); }
RSC_HD double rabs(double x) { return fabs(x); }
RSC_HD float rabs(float x) { return fabsf(x); }
template <typename T> RSC_HD void rswap(T& a, T& b) { T t = a; a = b; b = t; }

// Per-lane strided view of an LDS (or host) slab.
struct LaneMat {
    double* base;
    int stride;
    RSC_HD double& operator()(int e) const { return base[e * stride]; }
    RSC_HD double& at(int r, int c) const { return base[(r * 12 + c) * stride]; }
};

// ---------------------------------------------------------------------------------------------
// Eigen building blocks (Jacobi.h, MathFunctions.h)
// ---------------------------------------------------------------------------------------------
// The two helpers below are written with value selects instead of if/else: in a wave whose lanes
// hold different hypotheses both branches would execute (two divisions and a square root each);
// the selected operands feed the same operations, so the results are bit-identical to Eigen's.
template <typename S> RSC_HD S eig_hypot(S x, S y) {
    const S ax = rabs(x), ay = rabs(y);
    const bool gx = ax > ay;
    const S p = gx ? ax : ay;
    const S qp = (gx ? ay : ax) / p;  // in [0, 1] (p == 0 is overridden below)
    const S r = p * sqrt_unit(S(1) + qp * qp);
    return (p == S(0)) ? S(0) : r;
}

// JacobiRotation::makeGivens (real case).
// |t| <= 1, so 1 + t^2 is in [1, 2] and |u| in [1, sqrt 2] (the *_unit forms above).  The two special
// cases (p == 0; q == 0, which wins) are one select on values computed from p and q alone, so the
// chain after 1/u is a multiply and two selects.
template <typename S> RSC_HD void make_givens(S p, S q, S& c, S& s) {
    const bool big = rabs(p) > rabs(q);
    const S t = (big ? q : p) / (big ? p : q);
    S u = sqrt_unit(S(1) + t * t);
    if ((big ? p : q) < S(0)) u = -u;
    const S r = recip_unit(u);  // big: c = 1/u, s = -t*c;  else: s = -1/u (= -(1/u)), c = -t*s
    const S sb = -r;
    const S cc = big ? r : (-t) * sb;
    const S ss = big ? (-t) * r : sb;
    const bool qz = q == S(0), sp = (p == S(0)) | qz;
    const S c_sp = qz ? ((p < S(0)) ? S(-1) : S(1)) : S(0);
    const S s_sp = qz ? S(0) : ((q < S(0)) ? S(1) : S(-1));
    c = sp ? c_sp : cc;
    s = sp ? s_sp : ss;
}

// Ascending selection sort of the eigenvalues (end of computeFromTridiagonal_impl): the same
// comparisons and swaps as Eigen, recorded as a permutation (sorted column c = column perm[c]).
// Written with value selects only — conditional stores into the arrays would let LLVM merge the
// mutually exclusive swaps into one dynamically indexed store, forcing the arrays to scratch.
template <typename S, int n>
RSC_HD void eig_sort(S (&diag)[n], int (&perm)[n]) {
    RSC_UNROLL for (int i = 0; i < n - 1; ++i) {
        int kk = 0;
        S mn = diag[i];
        RSC_UNROLL for (int j = 1; j < n - i; ++j) {
            const bool lt = diag[i + j] < mn;
            mn = lt ? diag[i + j] : mn;
            kk = lt ? j : kk;
        }
        RSC_UNROLL for (int j = 1; j < n - i; ++j) {
            const bool sw = (j == kk);
            const S a = diag[i], b = diag[i + j];
            diag[i] = sw ? b : a;
            diag[i + j] = sw ? a : b;
            const int pa = perm[i], pb = perm[i + j];
            perm[i] = sw ? pb : pa;
            perm[i + j] = sw ? pa : pb;
        }
    }
}

// Optional hook of a QR rotation sink: `q.prefetch(k)` is called at the top of the chase slot k,
// before the Givens rotation is computed, so that a sink keeping Q in LDS issues the loads of
// columns k, k+1 while the chase runs (each slot is its own basic block; loads placed inside
// qapply are issued after the rotation and waited for at once, serialising the slots).
template <typename Q, typename = void>
struct qr_has_prefetch { static constexpr bool value = false; };
template <typename Q>
struct qr_has_prefetch<Q, decltype((void)std::declval<Q&>().prefetch(0))> { static constexpr bool value = true; };
// Optional hook `q.sweep_end()`: called after every implicit-QR step (once per loop iteration that
// ran a step, on the lanes that ran it), e.g. to publish the step's rotations to other waves.
template <typename Q, typename = void>
struct qr_has_sweep_end { static constexpr bool value = false; };
template <typename Q>
struct qr_has_sweep_end<Q, decltype((void)std::declval<Q&>().sweep_end())> { static constexpr bool value = true; };

// Implicit symmetric QR iterations on (diag, sub) with the rotations handed to
// `qapply(k, c, s, apply)` (which must perform Q = Q * G on columns k,k+1 when `apply`, and leave
// Q bit-identical otherwise).  computeFromTridiagonal_impl + sort.
// Returns Eigen's "Success".  perm: the sort's column permutation (identity when not converged,
// as Eigen skips the sort then); the caller applies it to its eigenvector storage.
// tridiag_qr reads diag[start], sub[start] by a select chain only when start > 0 (0: always).
#ifndef RSC_QR_START0
#define RSC_QR_START0 1
#endif
// How often tridiag_qr tests for a non-finite block (steps; 1 = every step).
#ifndef RSC_NAN_CHECK_EVERY
#define RSC_NAN_CHECK_EVERY 8
#endif
template <typename S, int n, typename QApply>
RSC_HD bool tridiag_qr(S (&diag)[n], S (&sub)[n - 1], QApply&& qapply, int (&perm)[n]) {
    const int maxIterations = 30;
    int end = n - 1, start = 0, iter = 0;
    const S considerAsZero = lim<S>::min();
    const S precision_inv = S(1) / lim<S>::eps();
    // Branch-free sweep bookkeeping.  Each `if` of Eigen's loop (deflation test, end/start
    // searches, shift cases, the chase's edge updates) compiled to a branch — a scalar branch when
    // the group's values are uniform, an exec-mask region otherwise — and the sweep's ~100 branches
    // cost more than its rotations (one 12x12 Refine chase: 156 rotations, 23 sweeps, 221 k shader
    // clocks, 3x the make_givens chains; tools/eig_probe.hip).  Here every test is a value select on
    // the same operands (same results, bit for bit); the only branches left are the loop exit and
    // the chase's per-slot range guard, which skips slots outside [start, end).  Conditions are
    // combined with the non-short-circuit & and | (a short-circuit || is a branch again).
    // Single-exit loop (Eigen's two `break`s folded into `run`): with several exits the CFG
    // structurizer nests the loop and every lane pays for the extra control flow.
    bool run = true;
    while (run) {
        // for (i = start; i < end; ++i): |sub| < considerAsZero, or (sub/eps)^2 <= |d_i| + |d_i+1|
        RSC_UNROLL for (int i = 0; i < n - 1; ++i) {
            const S scaled = precision_inv * sub[i];
            const bool z = (int)(rabs(sub[i]) < considerAsZero) | (int)(scaled * scaled <= (rabs(diag[i]) + rabs(diag[i + 1])));
            sub[i] = (z & (i >= start) & (i < end)) ? S(0) : sub[i];
        }
        // The two searches on a bit mask of the nonzero sub-diagonal entries (a find-last-set instead
        // of an 11-step select chain each):
        // while (end > 0 && sub[end-1] == 0) end--;  ->  end = 1 + last nonzero index below end, or 0
        unsigned nz = 0u;
        RSC_UNROLL for (int i = 0; i < n - 1; ++i) nz |= (sub[i] != S(0)) ? (1u << i) : 0u;
        const unsigned live = nz & ((1u << end) - 1u);
        end = live ? 32 - __builtin_clz(live) : 0;
        run = end > 0;
        iter = run ? iter + 1 : iter;
        run = run & (iter <= maxIterations * n);
        if (!run) continue;
        // start = end - 1; while (start > 0 && sub[start-1] != 0) start--;
        //   ->  start = 1 + last zero index below end - 1, or 0
        const unsigned zero = ~nz & ((1u << (end - 1)) - 1u);
        start = zero ? 32 - __builtin_clz(zero) : 0;
#ifndef RSC_NO_NAN_EXIT
        // Non-finite block (Q4: a coplanar sample's NaN control points): when diag[start..end] and
        // sub[start..end-1] are all NaN, no entry deflates and Eigen's loop runs to maxIterations*n
        // sweeps (360 at n = 12).  This sweep's rotations are all NaN (make_givens(NaN, NaN)), so it
        // turns Q's columns start..end into NaN; every later sweep maps that state onto itself
        // (NaN in, NaN out; the block cannot change: its sub-diagonal never reads 0).  Ending after
        // this sweep with Eigen's NoConvergence (no sort) therefore returns Eigen's final state.
        // The test runs on the first step and then every RSC_NAN_CHECK_EVERY-th: a dead block is a
        // fixed point of the sweep, so the sweeps it runs before the next test leave the state
        // as Eigen's (all running lanes are at the same step, so the branch is wave-uniform).
        if ((unsigned)(iter - 1) % (unsigned)RSC_NAN_CHECK_EVERY == 0u) {
            unsigned dnan = 0u, snan = 0u;
            RSC_UNROLL for (int i = 0; i < n; ++i) dnan |= (diag[i] != diag[i]) ? (1u << i) : 0u;
            RSC_UNROLL for (int i = 0; i < n - 1; ++i) snan |= (sub[i] != sub[i]) ? (1u << i) : 0u;
            const unsigned lo = (1u << start) - 1u;
            const unsigned blk_d = ((2u << end) - 1u) & ~lo, blk_s = ((1u << end) - 1u) & ~lo;
            const bool dead = ((dnan & blk_d) == blk_d) & ((snan & blk_s) == blk_s);
            iter = dead ? maxIterations * n : iter;  // the next loop test ends it, not converged
        }
#endif
        // ---- tridiagonal_qr_step(diag, sub, start, end) ----
        S dEm1 = S(0), dE = S(0), eE = S(0), dS = S(0), zS = S(0);
        RSC_UNROLL for (int j = 1; j < n; ++j) {
            const bool m = j == end;
            dEm1 = m ? diag[j - 1] : dEm1;
            dE = m ? diag[j] : dE;
            eE = m ? sub[j - 1] : eE;
        }
#if RSC_QR_START0
        // start is 0 until a sub-diagonal entry above the bottom block deflates: the select chain
        // runs behind a branch that a wave skips while none of its lanes has start > 0
        dS = diag[0];
        zS = sub[0];
        if (__builtin_expect(start != 0, 0)) {
            RSC_UNROLL for (int j = 1; j < n - 1; ++j) {
                const bool m = j == start;
                dS = m ? diag[j] : dS;
                zS = m ? sub[j] : zS;
            }
        }
#else
        RSC_UNROLL for (int j = 0; j < n - 1; ++j) {
            const bool m = j == start;
            dS = m ? diag[j] : dS;
            zS = m ? sub[j] : zS;
        }
#endif
        // Wilkinson shift; the three cases of Eigen are evaluated side by side and selected
        // (td == 0: mu - |e|; e^2 underflows: the two-quotient form; otherwise e^2/(td +- h))
        const S td = (dEm1 - dE) * S(0.5);
        const S e = eE;
        const S e2 = eE * eE;
        const S h = eig_hypot(td, e);
        const S mu_z = dE - rabs(e);
        const S mu_n = dE - e2 / (td + (td > S(0) ? h : -h));
        S mu = (td == S(0)) ? mu_z : mu_n;
        // e^2 underflowed (td != 0): the two-quotient form, behind a branch that a wave skips when
        // none of its lanes needs it (its two divisions are otherwise wasted on every step)
        if (__builtin_expect((td != S(0)) & (e2 == S(0)), 0))
            mu = dE - (e / (td + (td > S(0) ? S(1) : S(-1)))) * (e / h);
        S x = dS - mu;
        S z = zS;
        RSC_UNROLL for (int k = 0; k < n - 1; ++k) {
            if (k >= start && k < end) {
                if constexpr (qr_has_prefetch<QApply>::value) qapply.prefetch(k);
                S c, s;
                make_givens(x, z, c, s);
                S sdk = s * diag[k] + c * sub[k];
                S dkp1 = s * sub[k] + c * diag[k + 1];
                diag[k] = c * (c * diag[k] - s * sub[k]) - s * (c * sub[k] - s * diag[k + 1]);
                diag[k + 1] = s * sdk + c * dkp1;
                sub[k] = c * sdk - s * dkp1;
                if (k > 0) sub[k - 1] = (k > start) ? c * sub[k - 1] - s * z : sub[k - 1];
                x = sub[k];
                if (k < n - 2) {
                    const bool m = k < end - 1;
                    z = m ? -s * sub[k + 1] : z;
                    sub[k + 1] = m ? c * sub[k + 1] : sub[k + 1];
                }
                // Eigen skips identity rotations; qapply receives the flag and selects (a
                // conditional call here gets tail-duplicated into the loop latch, which turns
                // the QR loop into a nested loop that serialises the lanes of a wave)
                qapply(k, c, s, !(c == S(1) && s == S(0)));
            }
        }
        if constexpr (qr_has_sweep_end<QApply>::value) qapply.sweep_end();
        RSC_LOOP_FENCE();
    }
    const bool ok = (iter <= maxIterations * n);
#ifdef RSC_QR_STATS
    rsc_qr_stats_hook(n, iter);  // host-side diagnostics only (tools/)
#endif
    RSC_UNROLL for (int i = 0; i < n; ++i) perm[i] = i;
    if (ok) eig_sort<S, n>(diag, perm);
    return ok;
}

// Householder reflector of a register vector v[0..len) (MatrixBase::makeHouseholder).
template <typename S, int len>
RSC_HD void make_householder(S (&v)[len], S& tau, S& beta) {
    S tail = S(0);
    if (len > 1) {
        tail = v[1] * v[1];
        RSC_UNROLL for (int k = 2; k < len; ++k) tail = tail + v[k] * v[k];
    }
    S c0 = v[0];
    if (tail <= lim<S>::min()) {
        tau = S(0);
        beta = c0;
        RSC_UNROLL for (int k = 1; k < len; ++k) v[k] = S(0);
    } else {
        beta = rsqrt_(c0 * c0 + tail);
        if (c0 >= S(0)) beta = -beta;
        S den = c0 - beta;
        RSC_UNROLL for (int k = 1; k < len; ++k) v[k] = v[k] / den;
        tau = (beta - c0) / beta;
    }
}

// ---------------------------------------------------------------------------------------------
// SelfAdjointEigenSolver<Matrix<S,n,n>>::compute, register version (n = 3 or 4).
// A: lower triangle read.  V: eigenvectors in columns (ascending).  Returns "Success".
// ---------------------------------------------------------------------------------------------
template <typename S, int n>
RSC_HD bool sym_eig_reg(const S (&A)[n][n], S (&V)[n][n], S (&w)[n]) {
    S mat[n][n];
    RSC_UNROLL for (int i = 0; i < n; ++i)
        RSC_UNROLL for (int j = 0; j < n; ++j) mat[i][j] = (i >= j) ? A[i][j] : S(0);
    S scale = rabs(mat[0][0]);
    RSC_UNROLL for (int j = 0; j < n; ++j)
        RSC_UNROLL for (int i = 0; i < n; ++i) {
            if (i == 0 && j == 0) continue;
            S v = rabs(mat[i][j]);
            if (v > scale) scale = v;
        }
    if (scale == S(0)) scale = S(1);
    RSC_UNROLL for (int j = 0; j < n; ++j)
        RSC_UNROLL for (int i = j; i < n; ++i) mat[i][j] = mat[i][j] / scale;
    S diag[n], sub[n - 1];
    if (n == 3) {
        diag[0] = mat[0][0];
        S v1norm2 = mat[2][0] * mat[2][0];
        if (v1norm2 <= lim<S>::min()) {
            diag[1] = mat[1][1];
            diag[2] = mat[2][2];
            sub[0] = mat[1][0];
            sub[1] = mat[2][1];
            RSC_UNROLL for (int i = 0; i < n; ++i)
                RSC_UNROLL for (int j = 0; j < n; ++j) V[i][j] = (i == j) ? S(1) : S(0);
        } else {
            S beta = rsqrt_(mat[1][0] * mat[1][0] + v1norm2);
            S invBeta = S(1) / beta;
            S m01 = mat[1][0] * invBeta;
            S m02 = mat[2][0] * invBeta;
            S q = S(2) * m01 * mat[2][1] + m02 * (mat[2][2] - mat[1][1]);
            diag[1] = mat[1][1] + m02 * q;
            diag[2] = mat[2][2] - m02 * q;
            sub[0] = beta;
            sub[1] = mat[2][1] - m01 * q;
            V[0][0] = S(1); V[0][1] = S(0); V[0][2] = S(0);
            V[1][0] = S(0); V[1][1] = m01;  V[1][2] = m02;
            V[2][0] = S(0); V[2][1] = m02;  V[2][2] = -m01;
        }
    } else {
        S hC[n];
        RSC_UNROLL for (int i = 0; i < n - 1; ++i) {
            const int rs = n - i - 1;
            S v[n], hc[n], w2[n];
            RSC_UNROLL for (int k = 0; k < n; ++k) v[k] = S(0);
            RSC_UNROLL for (int k = 0; k < n; ++k) if (k < rs) v[k] = mat[i + 1 + k][i];
            // makeHouseholder on v[0..rs)
            S tail = S(0);
            if (rs > 1) {
                tail = v[1] * v[1];
                RSC_UNROLL for (int k = 2; k < n; ++k) if (k < rs) tail = tail + v[k] * v[k];
            }
            S c0 = v[0], h, beta;
            if (tail <= lim<S>::min()) {
                h = S(0);
                beta = c0;
                RSC_UNROLL for (int k = 1; k < n; ++k) if (k < rs) v[k] = S(0);
            } else {
                beta = rsqrt_(c0 * c0 + tail);
                if (c0 >= S(0)) beta = -beta;
                S den = c0 - beta;
                RSC_UNROLL for (int k = 1; k < n; ++k) if (k < rs) v[k] = v[k] / den;
                h = (beta - c0) / beta;
            }
            v[0] = S(1);
            RSC_UNROLL for (int k = 1; k < n; ++k) if (k < rs) mat[i + 1 + k][i] = v[k];
            RSC_UNROLL for (int k = 0; k < n; ++k) w2[k] = h * v[k];
            RSC_UNROLL for (int k = 0; k < n; ++k) {
                if (k < rs) {
                    S acc = S(0);
                    RSC_UNROLL for (int m = 0; m < n; ++m) {
                        if (m < rs) {
                            const int r = i + 1 + k, c = i + 1 + m;
                            S a = (r >= c) ? mat[r][c] : mat[c][r];
                            acc = (m == 0) ? a * w2[m] : acc + a * w2[m];
                        }
                    }
                    hc[k] = acc;
                }
            }
            S dot = hc[0] * v[0];
            RSC_UNROLL for (int k = 1; k < n; ++k) if (k < rs) dot = dot + hc[k] * v[k];
            S alpha = (h * S(-0.5)) * dot;
            RSC_UNROLL for (int k = 0; k < n; ++k) if (k < rs) hc[k] = hc[k] + alpha * v[k];
            RSC_UNROLL for (int c = 0; c < n; ++c) {
                if (c < rs) {
                    S s1 = -v[c], s2 = -hc[c];
                    RSC_UNROLL for (int r = 0; r < n; ++r)
                        if (r >= c && r < rs) {
                            S& a = mat[i + 1 + r][i + 1 + c];
                            a = a + (s1 * hc[r] + s2 * v[r]);
                        }
                }
            }
            mat[i + 1][i] = beta;
            hC[i] = h;
        }
        RSC_UNROLL for (int k = 0; k < n; ++k) diag[k] = mat[k][k];
        RSC_UNROLL for (int k = 0; k < n - 1; ++k) sub[k] = mat[k + 1][k];
        // Householder sequence evalTo, in place (diag=1, strictly upper=0, reverse application)
        RSC_UNROLL for (int i = 0; i < n; ++i) {
            mat[i][i] = S(1);
            RSC_UNROLL for (int j = 0; j < n; ++j) if (j > i) mat[i][j] = S(0);
        }
        RSC_UNROLL for (int k = n - 2; k >= 0; --k) {
            const int cs = n - k - 1, b0 = k + 1;
            const S tau = hC[k];
            if (cs == 1) {
                mat[b0][b0] = mat[b0][b0] * (S(1) - tau);
            } else if (tau != S(0)) {
                S tmp[n];
                RSC_UNROLL for (int c = 0; c < n; ++c) {
                    if (c < cs) {
                        S acc = mat[k + 2][k] * mat[b0 + 1][b0 + c];
                        RSC_UNROLL for (int r = 1; r < n; ++r)
                            if (r < cs - 1) acc = acc + mat[k + 2 + r][k] * mat[b0 + 1 + r][b0 + c];
                        tmp[c] = acc + mat[b0][b0 + c];
                    }
                }
                RSC_UNROLL for (int c = 0; c < n; ++c) if (c < cs) mat[b0][b0 + c] = mat[b0][b0 + c] - tau * tmp[c];
                RSC_UNROLL for (int r = 0; r < n; ++r) {
                    if (r < cs - 1) {
                        S te = tau * mat[k + 2 + r][k];
                        RSC_UNROLL for (int c = 0; c < n; ++c)
                            if (c < cs) mat[b0 + 1 + r][b0 + c] = mat[b0 + 1 + r][b0 + c] - tmp[c] * te;
                    }
                }
            }
            RSC_UNROLL for (int r = 0; r < n; ++r) if (r > k) mat[r][k] = S(0);
        }
        RSC_UNROLL for (int i = 0; i < n; ++i)
            RSC_UNROLL for (int j = 0; j < n; ++j) V[i][j] = mat[i][j];
    }
    auto qapply = [&](int k, S c, S s, bool apply) {
        RSC_UNROLL for (int i = 0; i < n; ++i) {
            S xi = V[i][k], yi = V[i][k + 1];
            V[i][k] = apply ? c * xi - s * yi : xi;
            V[i][k + 1] = apply ? s * xi + c * yi : yi;
        }
    };
    int perm[n];
    bool ok = tridiag_qr<S, n>(diag, sub, qapply, perm);
    S Vs[n][n];
    RSC_UNROLL for (int r = 0; r < n; ++r)
        RSC_UNROLL for (int c = 0; c < n; ++c) {
            S x = V[r][0];
            RSC_UNROLL for (int p = 1; p < n; ++p) x = (perm[c] == p) ? V[r][p] : x;
            Vs[r][c] = x;
        }
    RSC_UNROLL for (int r = 0; r < n; ++r)
        RSC_UNROLL for (int c = 0; c < n; ++c) V[r][c] = Vs[r][c];
    RSC_UNROLL for (int i = 0; i < n; ++i) w[i] = diag[i] * scale;
    return ok;
}

// ---------------------------------------------------------------------------------------------
// 12x12 SelfAdjointEigenSolver::compute with the matrix in a per-lane LDS slab (LaneMat, row-major
// e = r*12 + c).  On entry the lower triangle holds MtM; on exit the slab holds the eigenvectors
// (columns, ascending eigenvalues).  Only the eigenvector matrix is needed by EPnP.
// ---------------------------------------------------------------------------------------------
// Part 1: scaling, Householder tridiagonalisation and accumulation of the Householder sequence
// into the slab.  Returns the scale; diag/sub receive the tridiagonal matrix.
RSC_HD double sym_eig12_tridiag(const LaneMat& M, double (&diag)[12], double (&sub)[11]) {
    constexpr int n = 12;
    // mat = lower triangle (upper zeroed); scale = max |.| in column-major order
    double scale = rabs(M.at(0, 0));
    RSC_UNROLL for (int j = 0; j < n; ++j)
        RSC_UNROLL for (int i = 0; i < n; ++i) {
            if (i < j) { M.at(i, j) = 0.0; continue; }
            if (i == 0 && j == 0) continue;
            double v = rabs(M.at(i, j));
            if (v > scale) scale = v;
        }
    if (scale == 0.0) scale = 1.0;
    RSC_UNROLL for (int j = 0; j < n; ++j)
        RSC_UNROLL for (int i = j; i < n; ++i) M.at(i, j) = M.at(i, j) / scale;

    double hC[n - 1];
    RSC_UNROLL for (int i = 0; i < n - 1; ++i) {
        constexpr int NN = n - 1;
        const int rs = n - i - 1;
        double v[NN], w2[NN], hc[NN];
        RSC_UNROLL for (int k = 0; k < NN; ++k) v[k] = (k < rs) ? M.at(i + 1 + k, i) : 0.0;
        double tail = 0.0;
        if (rs > 1) {
            tail = v[1] * v[1];
            RSC_UNROLL for (int k = 2; k < NN; ++k) if (k < rs) tail = tail + v[k] * v[k];
        }
        double c0 = v[0], h, beta;
        if (tail <= lim<double>::min()) {
            h = 0.0;
            beta = c0;
            RSC_UNROLL for (int k = 1; k < NN; ++k) if (k < rs) v[k] = 0.0;
        } else {
            beta = sqrt(c0 * c0 + tail);
            if (c0 >= 0.0) beta = -beta;
            double den = c0 - beta;
            RSC_UNROLL for (int k = 1; k < NN; ++k) if (k < rs) v[k] = v[k] / den;
            h = (beta - c0) / beta;
        }
        v[0] = 1.0;
        RSC_UNROLL for (int k = 1; k < NN; ++k) if (k < rs) M.at(i + 1 + k, i) = v[k];
        RSC_UNROLL for (int k = 0; k < NN; ++k) w2[k] = h * v[k];
        RSC_UNROLL for (int k = 0; k < NN; ++k) {
            if (k < rs) {
                double acc = 0.0;
                RSC_UNROLL for (int m = 0; m < NN; ++m) {
                    if (m < rs) {
                        const int r = i + 1 + k, c = i + 1 + m;
                        double a = (r >= c) ? M.at(r, c) : M.at(c, r);
                        acc = (m == 0) ? a * w2[m] : acc + a * w2[m];
                    }
                }
                hc[k] = acc;
            }
        }
        double dot = hc[0] * v[0];
        RSC_UNROLL for (int k = 1; k < NN; ++k) if (k < rs) dot = dot + hc[k] * v[k];
        double alpha = (h * -0.5) * dot;
        RSC_UNROLL for (int k = 0; k < NN; ++k) if (k < rs) hc[k] = hc[k] + alpha * v[k];
        RSC_UNROLL for (int c = 0; c < NN; ++c) {
            if (c < rs) {
                double s1 = -v[c], s2 = -hc[c];
                RSC_UNROLL for (int r = 0; r < NN; ++r)
                    if (r >= c && r < rs) {
                        double& a = M.at(i + 1 + r, i + 1 + c);
                        a = a + (s1 * hc[r] + s2 * v[r]);
                    }
            }
        }
        M.at(i + 1, i) = beta;
        hC[i] = h;
    }
    RSC_UNROLL for (int k = 0; k < n; ++k) diag[k] = M.at(k, k);
    RSC_UNROLL for (int k = 0; k < n - 1; ++k) sub[k] = M.at(k + 1, k);
    RSC_UNROLL for (int i = 0; i < n; ++i) {
        M.at(i, i) = 1.0;
        RSC_UNROLL for (int j = i + 1; j < n; ++j) M.at(i, j) = 0.0;
    }
    RSC_UNROLL for (int k = n - 2; k >= 0; --k) {
        const int cs = n - k - 1, b0 = k + 1;
        const double tau = hC[k];
        if (cs == 1) {
            M.at(b0, b0) = M.at(b0, b0) * (1.0 - tau);
        } else if (tau != 0.0) {
            double tmp[n - 1];
            RSC_UNROLL for (int c = 0; c < n - 1; ++c) {
                if (c < cs) {
                    double acc = M.at(k + 2, k) * M.at(b0 + 1, b0 + c);
                    RSC_UNROLL for (int r = 1; r < n - 1; ++r)
                        if (r < cs - 1) acc = acc + M.at(k + 2 + r, k) * M.at(b0 + 1 + r, b0 + c);
                    tmp[c] = acc + M.at(b0, b0 + c);
                }
            }
            RSC_UNROLL for (int c = 0; c < n - 1; ++c) if (c < cs) M.at(b0, b0 + c) = M.at(b0, b0 + c) - tau * tmp[c];
            RSC_UNROLL for (int r = 0; r < n - 1; ++r) {
                if (r < cs - 1) {
                    double te = tau * M.at(k + 2 + r, k);
                    RSC_UNROLL for (int c = 0; c < n - 1; ++c)
                        if (c < cs) M.at(b0 + 1 + r, b0 + c) = M.at(b0 + 1 + r, b0 + c) - tmp[c] * te;
                }
            }
        }
        RSC_UNROLL for (int r = k + 1; r < n; ++r) M.at(r, k) = 0.0;
    }
    return scale;
}

// Part 2: implicit symmetric QR on (diag, sub) accumulating the rotations into the slab's
// eigenvector matrix, then the ascending sort (columns 0..3 materialised).
RSC_HD bool sym_eig12_qr(const LaneMat& M, double (&diag)[12], double (&sub)[11]) {
    constexpr int n = 12;
    auto qapply = [&](int k, double c, double s, bool apply) {
        RSC_UNROLL for (int i = 0; i < n; ++i) {
            double xi = M.at(i, k), yi = M.at(i, k + 1);
            M.at(i, k) = apply ? c * xi - s * yi : xi;
            M.at(i, k + 1) = apply ? s * xi + c * yi : yi;
        }
    };
    int perm[n];
    const bool ok = tridiag_qr<double, n>(diag, sub, qapply, perm);
    // Only the eigenvector columns EPnP reads (0..3, the four smallest eigenvalues) are
    // materialised in sorted order; columns 4..11 keep the unsorted vectors (they are reused as
    // scratch for L_6x10 and rho).
    RSC_UNROLL for (int r = 0; r < n; ++r) {
        double v[4];
        RSC_UNROLL for (int c = 0; c < 4; ++c) v[c] = M.at(r, perm[c]);
        RSC_UNROLL for (int c = 0; c < 4; ++c) M.at(r, c) = v[c];
    }
    return ok;
}

RSC_HD bool sym_eig12(const LaneMat& M) {
    double diag[12], sub[11];
    sym_eig12_tridiag(M, diag, sub);
    return sym_eig12_qr(M, diag, sub);
}

// ---------------------------------------------------------------------------------------------
// JacobiSVD<MatrixXd>(A 6xk, ThinU|ThinV).solve(b) — see oracle/ora_linalg.h for the structure.
// ---------------------------------------------------------------------------------------------
#ifndef RSC_JSVD_STAMP
#define RSC_JSVD_STAMP(k, j) \
    do {                     \
    } while (0)
#endif
// LaneRows (device, a wave whose lanes all hold the same problem — the Refine's beta waves): U and V
// are not replicated; lane r keeps row r of U (r < 6) and of V (r < k) and applies each Jacobi
// rotation to its own row (2 products + 1 sum per matrix instead of 6 + 5 rows per lane), the rows
// gathered with readlane for the final solve.  Same operations on the same operands per entry, so
// the result is bit-identical to the replicated form.
#if defined(__HIP_DEVICE_COMPILE__)
__device__ __forceinline__ double lane_read(double v, int lane) {
    const int lo = __builtin_amdgcn_readlane(__double2loint(v), lane);
    const int hi = __builtin_amdgcn_readlane(__double2hiint(v), lane);
    return __hiloint2double(hi, lo);
}
#endif
template <int k, bool LaneRows = false>
RSC_HD void jacobi_svd_solve_6xk(const double (&Ain)[6][k], const double (&b)[6], double (&x)[k]) {
    constexpr int rows = 6;
    const double eps = lim<double>::eps();
    const double precision = 2.0 * eps;
    const double considerAsZero = lim<double>::min();
    double scale = rabs(Ain[0][0]);
    RSC_UNROLL for (int c = 0; c < k; ++c)
        RSC_UNROLL for (int r = 0; r < rows; ++r) {
            if (r == 0 && c == 0) continue;
            double v = rabs(Ain[r][c]);
            if (v > scale) scale = v;
        }
    if (scale == 0.0) scale = 1.0;
    double qr[rows][k];
    RSC_UNROLL for (int r = 0; r < rows; ++r)
        RSC_UNROLL for (int c = 0; c < k; ++c) qr[r][c] = Ain[r][c] / scale;
    double hCoeffs[k], nU[k], nD[k];
    int perm[k];
    RSC_UNROLL for (int c = 0; c < k; ++c) {
        double s = qr[0][c] * qr[0][c];
        RSC_UNROLL for (int r = 1; r < rows; ++r) s = s + qr[r][c] * qr[r][c];
        nD[c] = sqrt(s);
        nU[c] = nD[c];
        perm[c] = c;
    }
    const double ndt = sqrt(eps);
    RSC_UNROLL for (int kk = 0; kk < k; ++kk) {
        int big = kk;
        double bv = nU[kk];
        RSC_UNROLL for (int c = kk + 1; c < k; ++c)
            if (nU[c] > bv) { bv = nU[c]; big = c; }
        // transposition kk <-> big: swap columns, norms, and the permutation indices
        RSC_UNROLL for (int c = kk + 1; c < k; ++c) {
            if (c == big) {
                RSC_UNROLL for (int r = 0; r < rows; ++r) rswap(qr[r][kk], qr[r][c]);
                rswap(nU[kk], nU[c]);
                rswap(nD[kk], nD[c]);
                rswap(perm[kk], perm[c]);
            }
        }
        // Householder of qr[kk..5][kk]
        constexpr int L = rows;
        double v[L];
        RSC_UNROLL for (int r = 0; r < L; ++r) v[r] = 0.0;
        RSC_UNROLL for (int r = 0; r < L; ++r) if (r < rows - kk) v[r] = qr[kk + r][kk];
        double tail = 0.0;
        const int len = rows - kk;
        if (len > 1) {
            tail = v[1] * v[1];
            RSC_UNROLL for (int r = 2; r < L; ++r) if (r < len) tail = tail + v[r] * v[r];
        }
        double c0 = v[0], tau, beta;
        if (tail <= considerAsZero) {
            tau = 0.0;
            beta = c0;
            RSC_UNROLL for (int r = 1; r < L; ++r) if (r < len) v[r] = 0.0;
        } else {
            beta = sqrt(c0 * c0 + tail);
            if (c0 >= 0.0) beta = -beta;
            double den = c0 - beta;
            RSC_UNROLL for (int r = 1; r < L; ++r) if (r < len) v[r] = v[r] / den;
            tau = (beta - c0) / beta;
        }
        hCoeffs[kk] = tau;
        qr[kk][kk] = beta;
        RSC_UNROLL for (int r = 1; r < L; ++r) if (r < len) qr[kk + r][kk] = v[r];
        const int bc = k - kk - 1;
        if (bc > 0 && tau != 0.0) {
            double tmp[k];
            RSC_UNROLL for (int c = 0; c < k; ++c) {
                if (c < bc) {
                    double acc = qr[kk + 1][kk] * qr[kk + 1][kk + 1 + c];
                    RSC_UNROLL for (int r = 2; r < rows; ++r)
                        if (r < len) acc = acc + qr[kk + r][kk] * qr[kk + r][kk + 1 + c];
                    tmp[c] = acc + qr[kk][kk + 1 + c];
                }
            }
            RSC_UNROLL for (int c = 0; c < k; ++c) if (c < bc) qr[kk][kk + 1 + c] = qr[kk][kk + 1 + c] - tau * tmp[c];
            RSC_UNROLL for (int r = 1; r < rows; ++r) {
                if (r < len) {
                    double te = tau * qr[kk + r][kk];
                    RSC_UNROLL for (int c = 0; c < k; ++c)
                        if (c < bc) qr[kk + r][kk + 1 + c] = qr[kk + r][kk + 1 + c] - tmp[c] * te;
                }
            }
        }
        RSC_UNROLL for (int j = kk + 1; j < k; ++j) {
            if (nU[j] != 0.0) {
                double temp = rabs(qr[kk][j]) / nU[j];
                temp = (1.0 + temp) * (1.0 - temp);
                temp = temp < 0.0 ? 0.0 : temp;
                double q = nU[j] / nD[j];
                double temp2 = temp * (q * q);
                if (temp2 <= ndt) {
                    double s = 0.0;
                    if (kk + 1 < rows) {
                        s = qr[kk + 1][j] * qr[kk + 1][j];
                        RSC_UNROLL for (int r = kk + 2; r < rows; ++r) s = s + qr[r][j] * qr[r][j];
                    }
                    nD[j] = sqrt(s);
                    nU[j] = nD[j];
                } else {
                    nU[j] *= sqrt(temp);
                }
            }
        }
    }
    RSC_JSVD_STAMP(k, 0);  // QR preconditioner done
    double W[k][k], U[rows][k], V[k][k];
    RSC_UNROLL for (int r = 0; r < k; ++r)
        RSC_UNROLL for (int c = 0; c < k; ++c) W[r][c] = (c >= r) ? qr[r][c] : 0.0;
    RSC_UNROLL for (int r = 0; r < rows; ++r)
        RSC_UNROLL for (int c = 0; c < k; ++c) U[r][c] = (r == c) ? 1.0 : 0.0;
    RSC_UNROLL for (int kk = k - 1; kk >= 0; --kk) {
        const double tau = hCoeffs[kk];
        const int len = rows - kk;
        if (tau != 0.0) {
            double tmp[k];
            RSC_UNROLL for (int c = 0; c < k; ++c) {
                double acc = qr[kk + 1][kk] * U[kk + 1][c];
                RSC_UNROLL for (int r = 2; r < rows; ++r) if (r < len) acc = acc + qr[kk + r][kk] * U[kk + r][c];
                tmp[c] = acc + U[kk][c];
            }
            RSC_UNROLL for (int c = 0; c < k; ++c) U[kk][c] = U[kk][c] - tau * tmp[c];
            RSC_UNROLL for (int r = 1; r < rows; ++r) {
                if (r < len) {
                    double te = tau * qr[kk + r][kk];
                    RSC_UNROLL for (int c = 0; c < k; ++c) U[kk + r][c] = U[kk + r][c] - tmp[c] * te;
                }
            }
        }
    }
    RSC_UNROLL for (int r = 0; r < k; ++r)
        RSC_UNROLL for (int c = 0; c < k; ++c) V[r][c] = (perm[c] == r) ? 1.0 : 0.0;
    // LaneRows: this lane's rows of U and V (lanes beyond 6 / k carry rows nobody reads)
    double Ur[k], Vr[k];
    if constexpr (LaneRows) {
#if defined(__HIP_DEVICE_COMPILE__)
        const int ln = (int)(threadIdx.x & 63u);
        RSC_UNROLL for (int c = 0; c < k; ++c) {
            double u = U[0][c], v = V[0][c];
            RSC_UNROLL for (int r = 1; r < rows; ++r) u = (ln == r) ? U[r][c] : u;
            RSC_UNROLL for (int r = 1; r < k; ++r) v = (ln == r) ? V[r][c] : v;
            Ur[c] = u;
            Vr[c] = v;
        }
#endif
    }

    RSC_JSVD_STAMP(k, 1);  // U formed
    double maxDiag = rabs(W[0][0]);
    RSC_UNROLL for (int i = 1; i < k; ++i) if (rabs(W[i][i]) > maxDiag) maxDiag = rabs(W[i][i]);
    bool finished = false;
    while (!finished) {
        finished = true;
        RSC_UNROLL for (int p = 1; p < k; ++p) {
            RSC_UNROLL for (int q = 0; q < p; ++q) {
                double pt = precision * maxDiag;
                double threshold = (considerAsZero < pt) ? pt : considerAsZero;
                if ((int)(rabs(W[p][q]) > threshold) | (int)(rabs(W[q][p]) > threshold)) {
                    finished = false;
                    // real_2x2_jacobi_svd.  Its inner ifs are value selects on the same operands
                    // (a divergent if is an exec-mask region, a uniform one a scalar branch; both cost
                    // more than the selects, tools/eig_probe.hip), and |tt| <= 1 puts tt^2 + 1 in
                    // [1, 2] and its root in [1, sqrt 2] (the short-chain *_unit forms).
                    double m00 = W[p][p], m01 = W[p][q], m10 = W[q][p], m11 = W[q][q];
                    const double t = m00 + m11;
                    const double d = m10 - m01;
                    const bool dz = rabs(d) < considerAsZero;
                    const double u = t / d;
                    const double tmp = sqrt(1.0 + u * u);
                    const double s1 = dz ? 0.0 : 1.0 / tmp;
                    const double c1 = dz ? 1.0 : u / tmp;
                    {
                        const bool rot = !((c1 == 1.0) & (s1 == 0.0));
                        const double x0 = m00, y0 = m10, x1 = m01, y1 = m11;
                        m00 = rot ? c1 * x0 + s1 * y0 : x0;
                        m10 = rot ? -s1 * x0 + c1 * y0 : y0;
                        m01 = rot ? c1 * x1 + s1 * y1 : x1;
                        m11 = rot ? -s1 * x1 + c1 * y1 : y1;
                    }
                    double cr, sr;
                    {
                        const double deno = 2.0 * rabs(m01);
                        const bool nz = deno < considerAsZero;
                        const double tau = (m00 - m11) / deno;
                        const double w = sqrt(tau * tau + 1.0);
                        const double tt = 1.0 / (tau > 0.0 ? tau + w : tau - w);
                        const double sign_t = tt > 0.0 ? 1.0 : -1.0;
                        const double nn = recip_unit(sqrt_unit(tt * tt + 1.0));
                        sr = nz ? 0.0 : -sign_t * (m01 / rabs(m01)) * rabs(tt) * nn;
                        cr = nz ? 1.0 : nn;
                    }
                    double crt = cr, srt = -sr;
                    double cl = c1 * crt - s1 * srt;
                    double sl = c1 * srt + s1 * crt;
                    if (!(cl == 1.0 && sl == 0.0)) {
                        RSC_UNROLL for (int c = 0; c < k; ++c) {
                            double xi = W[p][c], yi = W[q][c];
                            W[p][c] = cl * xi + sl * yi;
                            W[q][c] = -sl * xi + cl * yi;
                        }
                        if constexpr (LaneRows) {
                            const double xi = Ur[p], yi = Ur[q];
                            Ur[p] = cl * xi + sl * yi;
                            Ur[q] = -sl * xi + cl * yi;
                        } else {
                            RSC_UNROLL for (int r = 0; r < rows; ++r) {
                                double xi = U[r][p], yi = U[r][q];
                                U[r][p] = cl * xi + sl * yi;
                                U[r][q] = -sl * xi + cl * yi;
                            }
                        }
                    }
                    if (!(cr == 1.0 && sr == 0.0)) {
                        RSC_UNROLL for (int r = 0; r < k; ++r) {
                            double xi = W[r][p], yi = W[r][q];
                            W[r][p] = cr * xi - sr * yi;
                            W[r][q] = sr * xi + cr * yi;
                        }
                        if constexpr (LaneRows) {
                            const double xi = Vr[p], yi = Vr[q];
                            Vr[p] = cr * xi - sr * yi;
                            Vr[q] = sr * xi + cr * yi;
                        } else {
                            RSC_UNROLL for (int r = 0; r < k; ++r) {
                                double xi = V[r][p], yi = V[r][q];
                                V[r][p] = cr * xi - sr * yi;
                                V[r][q] = sr * xi + cr * yi;
                            }
                        }
                    }
                    double a = rabs(W[p][p]), bq = rabs(W[q][q]);
                    double mm = (a < bq) ? bq : a;
                    maxDiag = (maxDiag < mm) ? mm : maxDiag;
                }
            }
        }
        RSC_LOOP_FENCE();
    }
    RSC_JSVD_STAMP(k, 2);  // Jacobi sweeps done
    if constexpr (LaneRows) {  // rows back from their lanes (uniform values) for the sort and solve
#if defined(__HIP_DEVICE_COMPILE__)
        RSC_UNROLL for (int c = 0; c < k; ++c) {
            RSC_UNROLL for (int r = 0; r < rows; ++r) U[r][c] = lane_read(Ur[c], r);
            RSC_UNROLL for (int r = 0; r < k; ++r) V[r][c] = lane_read(Vr[c], r);
        }
#endif
    }
    double sv[k];
    RSC_UNROLL for (int i = 0; i < k; ++i) {
        double a = W[i][i];
        sv[i] = rabs(a);
        if (a < 0.0) RSC_UNROLL for (int r = 0; r < rows; ++r) U[r][i] = -U[r][i];
    }
    RSC_UNROLL for (int i = 0; i < k; ++i) sv[i] = sv[i] * scale;
    int nonzero = k;
    bool stop = false;
    RSC_UNROLL for (int i = 0; i < k; ++i) {
        if (!stop) {
            int pos = 0;
            double mv = sv[i];
            RSC_UNROLL for (int j = 1; j < k; ++j)
                if (j < k - i && sv[i + j] > mv) { mv = sv[i + j]; pos = j; }
            if (mv == 0.0) {
                nonzero = i;
                stop = true;
            } else if (pos) {
                RSC_UNROLL for (int j = 1; j < k; ++j) {
                    if (j == pos && i + j < k) {
                        rswap(sv[i], sv[i + j]);
                        RSC_UNROLL for (int r = 0; r < rows; ++r) rswap(U[r][i + j], U[r][i]);
                        RSC_UNROLL for (int r = 0; r < k; ++r) rswap(V[r][i + j], V[r][i]);
                    }
                }
            }
        }
    }
    double thr = sv[0] * ((double)k * eps);
    double premult = (thr < considerAsZero) ? considerAsZero : thr;
    // SVDBase::rank(): i = nonzero-1; while (i >= 0 && sv[i] < premult) --i;
    int i2 = nonzero - 1;
    RSC_UNROLL for (int t = k - 1; t >= 0; --t)
        if (t == i2 && sv[t] < premult) i2--;
    const int rank = i2 + 1;
    double tmpv[k];
    RSC_UNROLL for (int j = 0; j < k; ++j) {
        if (j < rank) {
            double acc = U[0][j] * b[0];
            RSC_UNROLL for (int r = 1; r < rows; ++r) acc = acc + U[r][j] * b[r];
            tmpv[j] = (1.0 / sv[j]) * acc;
        }
    }
    RSC_UNROLL for (int r = 0; r < k; ++r) {
        if (rank == 0) { x[r] = 0.0; continue; }
        double acc = V[r][0] * tmpv[0];
        RSC_UNROLL for (int j = 1; j < k; ++j) if (j < rank) acc = acc + V[r][j] * tmpv[j];
        x[r] = acc;
    }
}


// Matrix3d::inverse (cofactors); result(r,c) = cofactor(c,r) * invdet.
RSC_HD void inverse3(const double (&m)[3][3], double (&o)[3][3]) {
    double cof[3][3];
    RSC_UNROLL for (int i = 0; i < 3; ++i)
        RSC_UNROLL for (int j = 0; j < 3; ++j) {
            const int i1 = (i + 1) % 3, i2 = (i + 2) % 3, j1 = (j + 1) % 3, j2 = (j + 2) % 3;
            cof[i][j] = m[i1][j1] * m[i2][j2] - m[i1][j2] * m[i2][j1];
        }
    double det = cof[0][0] * m[0][0] + cof[1][0] * m[1][0] + cof[2][0] * m[2][0];
    double invdet = 1.0 / det;
    RSC_UNROLL for (int r = 0; r < 3; ++r)
        RSC_UNROLL for (int c = 0; c < 3; ++c) o[r][c] = cof[c][r] * invdet;
}

template <typename S>
RSC_HD void quat_to_R(S w, S x, S y, S z, S (&R)[3][3]) {
    const S tx = S(2) * x, ty = S(2) * y, tz = S(2) * z;
    const S twx = tx * w, twy = ty * w, twz = tz * w;
    const S txx = tx * x, txy = ty * x, txz = tz * x;
    const S tyy = ty * y, tyz = tz * y, tzz = tz * z;
    R[0][0] = S(1) - (tyy + tzz); R[0][1] = txy - twz;          R[0][2] = txz + twy;
    R[1][0] = txy + twz;          R[1][1] = S(1) - (txx + tzz); R[1][2] = tyz - twx;
    R[2][0] = txz - twy;          R[2][1] = tyz + twx;          R[2][2] = S(1) - (txx + tyy);
}

RSC_HD double det3(const double (&m)[3][3]) {
    double h0 = m[0][0] * (m[1][1] * m[2][2] - m[1][2] * m[2][1]);
    double h1 = m[0][1] * (m[1][0] * m[2][2] - m[1][2] * m[2][0]);
    double h2 = m[0][2] * (m[1][0] * m[2][1] - m[1][1] * m[2][0]);
    return h0 - h1 + h2;
}

// ---------------------------------------------------------------------------------------------
// glibc TYPE_3 rand() stream, jump-ahead form.  The generator is linear over Z/2^32:
//   r[i] = r[i-31] + r[i-3], output = r >> 1.
// A problem's stream position is a 31-word window w = (r[m-31], ..., r[m-1]); the g-th next raw
// word is r[m+g] = sum_j T[g][j] * w[j] (mod 2^32) with T built on the host (rsc_rng_table).
// ---------------------------------------------------------------------------------------------
RSC_HD uint32_t rng_word(const uint32_t* __restrict__ T /* [g][32] */, const uint32_t (&w)[31], int g) {
    const uint32_t* t = T + (size_t)g * 32;
    uint32_t acc = 0;
    RSC_UNROLL for (int j = 0; j < 31; ++j) acc += t[j] * w[j];
    return acc;
}

// DUtils::Random::RandomInt(0, size-1) given the raw word.
RSC_HD int random_index(uint32_t word, int size) {
    const int32_t r = (int32_t)(word >> 1);
    return int(((double)r / ((double)2147483647 + 1.0)) * size);
}

// Swap-remove sampling of `ms` indices over [0,N) from a fresh index list (PnPsolver.cpp:125-138).
template <int MAXS>
RSC_HD void swap_remove_sample(const uint32_t* words, int ms, int N, int (&out)[MAXS]) {
    int pos[MAXS], val[MAXS];
    int nmod = 0;
    RSC_UNROLL for (int i = 0; i < MAXS; ++i) {
        if (i < ms) {
            const int size = N - i;
            const int randi = random_index(words[i], size);
            auto lookup = [&](int p) {
                int v = p;
                RSC_UNROLL for (int t = 0; t < MAXS; ++t)
                    if (t < nmod && pos[t] == p) v = val[t];
                return v;
            };
            const int idx = lookup(randi);
            out[i] = idx;
            const int back = lookup(size - 1);
            bool found = false;
            RSC_UNROLL for (int t = 0; t < MAXS; ++t)
                if (t < nmod && pos[t] == randi) { val[t] = back; found = true; }
            if (!found) {
                RSC_UNROLL for (int t = 0; t < MAXS; ++t)
                    if (t == nmod) { pos[t] = randi; val[t] = back; }
                nmod++;
            }
        }
    }
}

// ---------------------------------------------------------------------------------------------
// PnPsolver::CheckInliers for one correspondence (PnPsolver.cpp:245-266): float rotation,
// float reciprocal, projection in double rounded to float, float squared error, strict '<'.
// ---------------------------------------------------------------------------------------------
RSC_HD bool pnp_inlier(const float (&R)[9], const float (&t)[3], double fx, double fy, double cx, double cy,
                       float X, float Y, float Z, float u, float v, float maxErr) {
    // mRi*p3Dw + mti (:250): Matrix3f * Vector3f, coefficient-path reductions
    float Xc = ered3(R[0] * X, R[1] * Y, R[2] * Z) + t[0];
    float Yc = ered3(R[3] * X, R[4] * Y, R[5] * Z) + t[1];
    float Zc = ered3(R[6] * X, R[7] * Y, R[8] * Z) + t[2];
    float invZc = 1.0f / Zc;
    float ue = (float)(cx + fx * (double)Xc * (double)invZc);
    float ve = (float)(cy + fy * (double)Yc * (double)invZc);
    float du = ue - u, dv = ve - v;
    float e2 = du * du + dv * dv;
    return e2 < maxErr;
}

}  // namespace rsc
