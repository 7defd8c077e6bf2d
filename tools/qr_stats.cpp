// qr_stats — host diagnostic: implicit-QR sweep structure of the 12x12 EPnP eigenproblem on
// config-2 shaped hypotheses, and the rotation slots a wave executes when G hypotheses share it
// (the predicated, unrolled k-loop of tridiag_qr runs the union of the lanes' [start, end)).
// Build: g++ -O2 -std=c++17 -ffp-contract=off -I../orb-slam2-optimized_amd/csrc qr_stats.cpp
#include <algorithm>
#include <cstdio>
#include <random>
#include <vector>
#include "rsc_epnp.h"

using namespace rsc;

int main() {
    const int n = 2000, H = 19200;
    const double fx = 435.2046959714599, cx = 367.4517211914062, cy = 252.2008514404297;
    std::mt19937_64 g(7);
    std::uniform_real_distribution<double> U(0, 1);
    std::vector<float> P(3 * n), Q(2 * n);
    for (int i = 0; i < n; ++i) {
        const double u = 752 * U(g), v = 480 * U(g), d = 0.5 + 7.5 * U(g);
        P[3 * i] = (float)((u - cx) / fx * d); P[3 * i + 1] = (float)((v - cy) / fx * d); P[3 * i + 2] = (float)d;
        const bool in = U(g) < 0.4;
        Q[2 * i] = (float)(in ? u + U(g) - 0.5 : 752 * U(g));
        Q[2 * i + 1] = (float)(in ? v + U(g) - 0.5 : 480 * U(g));
    }
    std::vector<std::vector<std::pair<int, int>>> sweeps(H);  // per hypothesis: (start, end) per sweep
    std::vector<int> rot(H);
    std::uniform_int_distribution<int> pick(0, n - 1);
    for (int h = 0; h < H; ++h) {
        HypStore<4> st;
        int idx[4];
        for (int k = 0; k < 4; ++k) {
            bool dup;
            do { idx[k] = pick(g); dup = false; for (int j = 0; j < k; ++j) dup |= idx[j] == idx[k]; } while (dup);
            for (int c = 0; c < 3; ++c) st.pw_[k][c] = P[3 * idx[k] + c];
            st.u_[k][0] = Q[2 * idx[k]]; st.u_[k][1] = Q[2 * idx[k] + 1];
        }
        st.rows_ = 4; st.spw = nullptr; st.sal = nullptr;
        const Intrinsics K{fx, fx, cx, cy};
        double cws[4][3];
        control_points_and_alphas(st, cws);
        double slab[160];
        LaneMat S{slab, 1};
        build_MtM(st, K, S);
        double diag[12], sub[11];
        sym_eig12_tridiag(S, diag, sub);
        int last = 100, s0 = 0;
        auto& sw = sweeps[h];
        auto qapply = [&](int k, double, double, bool) {
            if (k <= last) { if (last != 100) sw.push_back({s0, last + 1}); s0 = k; }
            last = k;
            rot[h]++;
        };
        int perm[12];
        tridiag_qr<double, 12>(diag, sub, qapply, perm);
        if (last != 100) sw.push_back({s0, last + 1});
    }
    double sw_mean = 0, rot_mean = 0;
    for (int h = 0; h < H; ++h) { sw_mean += sweeps[h].size(); rot_mean += rot[h]; }
    printf("per hypothesis: sweeps %.2f, rotations %.2f\n", sw_mean / H, rot_mean / H);
    for (int G : {1, 4, 16, 20, 64}) {
        double slots = 0, sweeps_w = 0, maxrot = 0, maxev = 0;
        for (int w = 0; w < H; w += G) {
            size_t ns = 0;
            double mr = 0;
            double me = 0;
            for (int l = 0; l < G; ++l) {
                ns = std::max(ns, sweeps[w + l].size());
                mr = std::max(mr, (double)rot[w + l]);
                me = std::max(me, (double)(rot[w + l] + sweeps[w + l].size() + 1));  // event form: rotations + setups
            }
            maxev += me;
            for (size_t i = 0; i < ns; ++i) {
                int lo = 99, hi = -1;
                for (int l = 0; l < G; ++l)
                    if (i < sweeps[w + l].size()) { lo = std::min(lo, sweeps[w + l][i].first); hi = std::max(hi, sweeps[w + l][i].second); }
                slots += hi - lo;
            }
            sweeps_w += ns;
            maxrot += mr;
        }
        const double nw = (double)H / G;
        printf("G=%2d lanes-hyps/wave: sweeps/wave %.2f  union slots/wave %.1f  max lane rotations %.1f  "
               "event form: max lane events %.1f\n", G, sweeps_w / nw, slots / nw, maxrot / nw, maxev / nw);
    }
    return 0;
}
