// qr_events.h — DIAGNOSTIC variants of the 12x12 implicit symmetric QR (not part of the product).
// Moved out of csrc/rsc_core.h: both forms are bit-identical to tridiag_qr<double, 12> and were
// measured slower on gfx950 (profiles/r02/qr_bench_variants_r2k.txt); they stay
// here for tools/qr_bench.hip, tools/quad_bench.hip and the host-emulation test of their equality.
#pragma once
#include "../orb-slam2-optimized_amd/csrc/rsc_core.h"

namespace rsc {

// ---------------------------------------------------------------------------------------------
// tridiag_qr<double, 12> in EVENT form: the same operations on the same operands for every matrix
// (bit-identical diag, perm and Q), but the implicit-QR iteration is flattened into a sequence of
// events — a sweep setup (deflation bookkeeping + Wilkinson shift) or ONE Givens rotation of the
// chase — so lanes that hold different matrices advance independently: a wave pays the max over its
// lanes of (rotations + sweeps) instead of, per sweep, the union of the lanes' windows for as many
// sweeps as its slowest lane.  Every event runs exactly one division / square root / division chain
// (the shift's eig_hypot + quotient, or makeGivens' t, sqrt(1 + t^2), 1/u) with selected operands.
//   ds: diag[0..11] then sub[12..22], in memory shared by the lanes computing the same matrix
//   (LDS for a quad; identical values are written by all of them).
//   rows: the rotation sink, R rows of Q: load(r, col), store(r, col, v); Q = Q * G(k, k+1).
// Deflation tests run inside the sweep as soon as an entry is final (sub[k-1] after rotation k,
// sub[end-1] after the last one) — the values Eigen's scan at the next iteration reads; the zero
// pattern of sub is kept as a bit mask so the end/start searches are integer ops.
RSC_HD int rsc_msb(unsigned v) { return 31 - __builtin_clz(v); }

template <int R, class Rows>
RSC_HD bool tridiag_qr_events12(double* ds, Rows& rows, int (&perm)[12]) {
    constexpr int n = 12;
    const int maxIterations = 30;
    const double considerAsZero = lim<double>::min();
    const double precision_inv = 1.0 / lim<double>::eps();
    auto deflate = [&](double s, double d0, double d1) {
        if (rabs(s) < considerAsZero) return true;
        const double scaled = precision_inv * s;
        return scaled * scaled <= (rabs(d0) + rabs(d1));
    };
    unsigned zmask = 0;  // bit i: sub[i] == 0
    RSC_UNROLL for (int i = 0; i < n - 1; ++i) {  // the first iteration's scan over [0, n-1)
        if (deflate(ds[n + i], ds[i], ds[i + 1])) {
            ds[n + i] = 0.0;
            zmask |= 1u << i;
        }
    }
    int end = n - 1, start = 0, iter = 0, k = -1;  // k < 0: a sweep setup is the next event
    double x = 0.0, z = 0.0, dk = 0.0, sk = 0.0, dkm1 = 0.0, dnext = 0.0, snext = 0.0;
    double qx[R], qy[R];
    RSC_UNROLL for (int r = 0; r < R; ++r) qx[r] = qy[r] = 0.0;
    bool active = true;
    while (active) {
        const bool setup = k < 0;
        double td = 0.0, e = 0.0, dE = 0.0, dS = 0.0, zS = 0.0;
        if (setup) {
            const unsigned nz = ~zmask & ((1u << end) - 1u);  // while (end > 0 && sub[end-1] == 0) end--
            end = nz ? rsc_msb(nz) + 1 : 0;
            active = end > 0;
            if (active) {
                iter++;
                active = iter <= maxIterations * n;
            }
            if (active) {
                const unsigned zb = zmask & ((1u << (end - 1)) - 1u);  // while (start > 0 && sub[start-1] != 0)
                start = zb ? rsc_msb(zb) + 1 : 0;
                const double dEm1 = ds[end - 1];
                dE = ds[end];
                e = ds[n + end - 1];
                dS = ds[start];
                zS = ds[n + start];
                td = (dEm1 - dE) * 0.5;
            }
        }
        if (active) {
            // the event's chain: setup -> eig_hypot(td, e) and e^2 / (td +- h); rotation -> makeGivens(x, z)
            const double ax = rabs(td), ay = rabs(e);
            const bool gx = ax > ay;
            const double P = gx ? ax : ay;
            const bool big = rabs(x) > rabs(z);
            const double n1 = setup ? (gx ? ay : ax) : (big ? z : x);
            const double d1 = setup ? P : (big ? x : z);
            const double t = n1 / d1;
            const double sq = rsqrt_(1.0 + t * t);
            const double hh = (P == 0.0) ? 0.0 : P * sq;
            double u = sq;
            if ((big ? x : z) < 0.0) u = -u;
            const double e2 = e * e;
            const double q2 = (setup ? e2 : 1.0) / (setup ? td + (td > 0.0 ? hh : -hh) : u);
            if (setup) {
                double mu = dE;
                if (td == 0.0) {
                    mu -= rabs(e);
                } else if (e2 == 0.0) {
                    mu -= (e / (td + (td > 0.0 ? 1.0 : -1.0))) * (e / hh);
                } else {
                    mu -= q2;
                }
                x = dS - mu;
                z = zS;
                k = start;
                dk = dS;
                sk = zS;
                dnext = ds[k + 1];
                snext = (k < end - 1) ? ds[n + k + 1] : 0.0;
                RSC_UNROLL for (int r = 0; r < R; ++r) {
                    qx[r] = rows.load(r, k);
                    qy[r] = rows.load(r, k + 1);
                }
            } else {
                const double sb = -q2;  // makeGivens: r = 1/u
                double c = big ? q2 : (-t) * sb;
                double s = big ? (-t) * q2 : sb;
                if (x == 0.0) {
                    c = 0.0;
                    s = (z < 0.0) ? 1.0 : -1.0;
                }
                if (z == 0.0) {
                    c = (x < 0.0) ? -1.0 : 1.0;
                    s = 0.0;
                }
                const double dk1 = dnext;
                const double sdk = s * dk + c * sk;
                const double dkp1 = s * sk + c * dk1;
                const double dkn = c * (c * dk - s * sk) - s * (c * sk - s * dk1);
                const double dk1n = s * sdk + c * dkp1;
                const double skn = c * sdk - s * dkp1;
                ds[k] = dkn;
                if (k > start) {
                    const double skm1 = c * x - s * z;  // sub[k-1] is final: Eigen's next scan tests it
                    const bool zero = deflate(skm1, dkm1, dkn);
                    ds[n + k - 1] = zero ? 0.0 : skm1;
                    if (zero) zmask |= 1u << (k - 1);
                }
                x = skn;
                const bool more = k < end - 1;
                if (more) {
                    z = -s * snext;
                    sk = c * snext;
                }
                const bool apply = !(c == 1.0 && s == 0.0);  // Eigen skips identity rotations
                RSC_UNROLL for (int r = 0; r < R; ++r) {
                    const double a = qx[r], b = qy[r];
                    rows.store(r, k, apply ? c * a - s * b : a);
                    qx[r] = apply ? s * a + c * b : b;
                }
                dkm1 = dkn;
                dk = dk1n;
                if (more) {
                    k++;
                    dnext = ds[k + 1];
                    snext = (k < end - 1) ? ds[n + k + 1] : 0.0;
                    RSC_UNROLL for (int r = 0; r < R; ++r) qy[r] = rows.load(r, k + 1);
                } else {  // last rotation of the sweep: diag[end], sub[end-1] final
                    ds[k + 1] = dk1n;
                    RSC_UNROLL for (int r = 0; r < R; ++r) rows.store(r, k + 1, qx[r]);
                    const bool zero = deflate(skn, dkn, dk1n);
                    ds[n + k] = zero ? 0.0 : skn;
                    if (zero) zmask |= 1u << k;
                    k = -1;
                }
            }
        }
        RSC_LOOP_FENCE();
    }
    const bool ok = (iter <= maxIterations * n);
    double diag[n];
    RSC_UNROLL for (int i = 0; i < n; ++i) {
        diag[i] = ds[i];
        perm[i] = i;
    }
    if (ok) eig_sort<double, n>(diag, perm);
    return ok;
}

// ---------------------------------------------------------------------------------------------
// The event form split in two (the split-chase EPnP eigen-solver, rsc_quad.h):
//   QrChase12 — the Givens chase of tridiag_qr_events12 on (diag, sub) alone, as a resumable state
//     machine run by ONE lane per matrix, which hands every non-identity rotation (k, c, s) to a log
//     instead of applying it (Eigen skips identity rotations, so dropping them changes nothing);
//   QrRowApply — one row of Q replaying the log in order: Q = Q * G(k, k+1) per entry.  Rows of Q
//     are independent under right rotations, so any lanes may own any rows.  Within a sweep the
//     chase visits k, k+1, ... and the new column k+1 of one rotation is column "k" of the next, so
//     the row keeps it in a register (x) and touches memory once per entry: load b = row[k+1],
//     store row[k].  A new sweep (k != previous k + 1) first stores the pending value.
// Same operations on the same operands as tridiag_qr / tridiag_qr_events12: bit-identical.
// ds(i): accessor of diag[0..11] (i < 12) and sub[0..10] (i = 12 + j) of this lane's matrix.
struct QrChase12 {
    unsigned zmask;  // bit i: sub[i] == 0
    int end, start, iter, k;  // k < 0: a sweep setup is the next event
    double x, z, dk, sk, dkm1, dnext, snext;
    bool active;

    RSC_HD static bool deflate(double s, double d0, double d1) {
        if (rabs(s) < lim<double>::min()) return true;
        const double scaled = (1.0 / lim<double>::eps()) * s;
        return scaled * scaled <= (rabs(d0) + rabs(d1));
    }

    template <class DS>
    RSC_HD void init(DS&& ds) {
        zmask = 0;
        RSC_UNROLL for (int i = 0; i < 11; ++i) {  // the first iteration's scan over [0, n-1)
            if (deflate(ds(12 + i), ds(i), ds(i + 1))) {
                ds(12 + i) = 0.0;
                zmask |= 1u << i;
            }
        }
        end = 11;
        start = 0;
        iter = 0;
        k = -1;
        x = z = dk = sk = dkm1 = dnext = snext = 0.0;
        active = true;
    }

    RSC_HD bool converged() const { return iter <= 30 * 12; }

    // Runs events until the matrix is done or `cap` rotations have been logged; returns the number
    // logged.  log(e, k, c, s) records entry e.
    template <class DS, class Log>
    RSC_HD int run(DS&& ds, Log&& log, int cap) {
        constexpr int n = 12;
        int nl = 0;
        while (active && nl < cap) {
            const bool setup = k < 0;
            double td = 0.0, e = 0.0, dE = 0.0, dS = 0.0, zS = 0.0;
            if (setup) {
                const unsigned nz = ~zmask & ((1u << end) - 1u);  // while (end > 0 && sub[end-1] == 0) end--
                end = nz ? rsc_msb(nz) + 1 : 0;
                active = end > 0;
                if (active) {
                    iter++;
                    active = iter <= 30 * n;
                }
                if (active) {
                    const unsigned zb = zmask & ((1u << (end - 1)) - 1u);  // while (start > 0 && sub[start-1] != 0)
                    start = zb ? rsc_msb(zb) + 1 : 0;
                    const double dEm1 = ds(end - 1);
                    dE = ds(end);
                    e = ds(n + end - 1);
                    dS = ds(start);
                    zS = ds(n + start);
                    td = (dEm1 - dE) * 0.5;
                }
            }
            if (active) {
                // setup -> eig_hypot(td, e) and e^2 / (td +- h); rotation -> makeGivens(x, z)
                const double ax = rabs(td), ay = rabs(e);
                const bool gx = ax > ay;
                const double P = gx ? ax : ay;
                const bool big = rabs(x) > rabs(z);
                const double n1 = setup ? (gx ? ay : ax) : (big ? z : x);
                const double d1 = setup ? P : (big ? x : z);
                const double t = n1 / d1;
                const double sq = rsqrt_(1.0 + t * t);
                const double hh = (P == 0.0) ? 0.0 : P * sq;
                double u = sq;
                if ((big ? x : z) < 0.0) u = -u;
                const double e2 = e * e;
                const double q2 = (setup ? e2 : 1.0) / (setup ? td + (td > 0.0 ? hh : -hh) : u);
                if (setup) {
                    double mu = dE;
                    if (td == 0.0) {
                        mu -= rabs(e);
                    } else if (e2 == 0.0) {
                        mu -= (e / (td + (td > 0.0 ? 1.0 : -1.0))) * (e / hh);
                    } else {
                        mu -= q2;
                    }
                    x = dS - mu;
                    z = zS;
                    k = start;
                    dk = dS;
                    sk = zS;
                    dnext = ds(k + 1);
                    snext = (k < end - 1) ? ds(n + k + 1) : 0.0;
                } else {
                    const double sb = -q2;  // makeGivens: r = 1/u
                    double c = big ? q2 : (-t) * sb;
                    double s = big ? (-t) * q2 : sb;
                    if (x == 0.0) {
                        c = 0.0;
                        s = (z < 0.0) ? 1.0 : -1.0;
                    }
                    if (z == 0.0) {
                        c = (x < 0.0) ? -1.0 : 1.0;
                        s = 0.0;
                    }
                    const double dk1 = dnext;
                    const double sdk = s * dk + c * sk;
                    const double dkp1 = s * sk + c * dk1;
                    const double dkn = c * (c * dk - s * sk) - s * (c * sk - s * dk1);
                    const double dk1n = s * sdk + c * dkp1;
                    const double skn = c * sdk - s * dkp1;
                    ds(k) = dkn;
                    if (k > start) {
                        const double skm1 = c * x - s * z;  // sub[k-1] is final: Eigen's next scan tests it
                        const bool zero = deflate(skm1, dkm1, dkn);
                        ds(n + k - 1) = zero ? 0.0 : skm1;
                        if (zero) zmask |= 1u << (k - 1);
                    }
                    x = skn;
                    const bool more = k < end - 1;
                    if (more) {
                        z = -s * snext;
                        sk = c * snext;
                    }
                    if (!(c == 1.0 && s == 0.0)) {
                        log(nl, k, c, s);
                        nl++;
                    }
                    dkm1 = dkn;
                    dk = dk1n;
                    if (more) {
                        k++;
                        dnext = ds(k + 1);
                        snext = (k < end - 1) ? ds(n + k + 1) : 0.0;
                    } else {  // last rotation of the sweep: diag[end], sub[end-1] final
                        ds(k + 1) = dk1n;
                        const bool zero = deflate(skn, dkn, dk1n);
                        ds(n + k) = zero ? 0.0 : skn;
                        if (zero) zmask |= 1u << k;
                        k = -1;
                    }
                }
            }
            RSC_LOOP_FENCE();
        }
        return nl;
    }
};

struct QrRowApply {
    int pk = -8;   // k of the previous entry (< 0: none yet)
    double x = 0;  // pending value of row[pk + 1]
    // row: pointer to the 12 entries of the row (any memory)
    RSC_HD void step(double* row, int k, double c, double s) {
        const bool cont = (k == pk + 1);
        if (!cont && pk >= 0) row[pk + 1] = x;
        const double a = cont ? x : row[k];
        const double b = row[k + 1];
        row[k] = c * a - s * b;
        x = s * a + c * b;
        pk = k;
    }
    RSC_HD void flush(double* row) {
        if (pk >= 0) row[pk + 1] = x;
        pk = -8;
    }
};

}  // namespace rsc
