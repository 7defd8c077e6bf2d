// Drives the C++ facade (PnPsolver / Sim3Solver templates) with mock Frame / KeyFrame / MapPoint
// types built from a binary scene file written by tests/test_gpu_facade.py, and writes every
// iterate() result back for comparison with the oracle.  Runs on the GPU box.
#include <cstdio>
#include <cstdint>
#include <cstring>
#include <memory>
#include <vector>
#include "PnPsolver.hpp"
#include "Sim3Solver.hpp"
#include "Optimizer.hpp"
#include "MLPnPsolver.hpp"
#include "ORBmatcher.hpp"
#include "KeyFrameDatabase.hpp"
#include <map>
#include <set>

struct Vec3 { float v[3]; float operator()(int i) const { return v[i]; } float& operator()(int i) { return v[i]; } };
struct Mat3 { float m[3][3]; float operator()(int r, int c) const { return m[r][c]; } float& operator()(int r, int c) { return m[r][c]; } };
struct Mat4 { float m[4][4]; float& operator()(int r, int c) { return m[r][c]; } float operator()(int r, int c) const { return m[r][c]; } };
struct Pt { float x, y; };
struct KeyPoint { Pt pt; int octave; float angle = 0.f; };
struct Frame { std::vector<KeyPoint> mvKeysUn; std::vector<float> mvLevelSigma2; float fx, fy, cx, cy; };
struct KeyFrame;
struct MapPoint {
    bool bad = false; Vec3 X; int idx1 = -1, idx2 = -1; KeyFrame* kf1 = nullptr;
    bool isBad() const { return bad; }
    Vec3 GetWorldPos() const { return X; }
    int GetIndexInKeyFrame(const std::shared_ptr<KeyFrame>& kf) const;
};
struct KeyFrame {
    std::vector<KeyPoint> mvKeysUn; std::vector<float> mvLevelSigma2, mvInvLevelSigma2; Mat3 mK; Mat3 R; Vec3 t;
    std::vector<std::shared_ptr<MapPoint>> mps;
    std::vector<std::shared_ptr<MapPoint>> GetMapPointMatches() { return mps; }
    Mat3 GetRotation() const { return R; }
    Vec3 GetTranslation() const { return t; }
};
int MapPoint::GetIndexInKeyFrame(const std::shared_ptr<KeyFrame>& kf) const { return kf.get() == kf1 ? idx1 : idx2; }

// cv::Mat stand-in for descriptor rows (mDescriptors.ptr<uint8_t>(i)) and the SearchByBoW views
struct DescMat {
    std::vector<uint8_t> d;
    template <class T> const T* ptr(int row) const { return reinterpret_cast<const T*>(d.data() + 32 * (size_t)row); }
};
using FeatVec = std::map<unsigned int, std::vector<unsigned int>>;
struct BowKF {
    int N = 0; DescMat mDescriptors; std::vector<KeyPoint> mvKeysUn; FeatVec mFeatVec;
    std::vector<std::shared_ptr<MapPoint>> mps;
    std::vector<std::shared_ptr<MapPoint>> GetMapPointMatches() const { return mps; }
};
struct BowFrame { int N = 0; DescMat mDescriptors; std::vector<KeyPoint> mvKeys; FeatVec mFeatVec; };

// g2o::Sim3 stand-in: rotation().coeffs()[k] (x, y, z, w), translation()[k], scale() as references
struct MockSim3 {
    struct V4 { double v[4]; double& operator[](int i) { return v[i]; } };
    struct Q { V4 c; V4& coeffs() { return c; } };
    struct V3d { double v[3]; double& operator[](int i) { return v[i]; } };
    Q q; V3d tr; double s = 1.0;
    Q& rotation() { return q; }
    V3d& translation() { return tr; }
    double& scale() { return s; }
};

// SearchBySim3 mocks: KeyFrame with the public members ORBmatcher::SearchBySim3 reads plus the
// GetGrid() getter, MapPoint with GetMaxDistance()/GetMinDistance()
struct S3KF;
struct S3MP {
    bool bad = false; Vec3 X; DescMat d; float dmax = 0, dmin = 0; const S3KF* home = nullptr; int idx = -1;
    bool isBad() const { return bad; }
    Vec3 GetWorldPos() const { return X; }
    DescMat GetDescriptor() const { return d; }
    float GetMaxDistance() const { return dmax; }
    float GetMinDistance() const { return dmin; }
    int GetIndexInKeyFrame(const std::shared_ptr<S3KF>& kf) const { return kf.get() == home ? idx : -1; }
};
struct S3KF {
    int N = 0; std::vector<KeyPoint> mvKeysUn; DescMat mDescriptors;
    int mnMinX = 0, mnMinY = 0, mnMaxX = 0, mnMaxY = 0;
    float mfGridElementWidthInv = 0, mfGridElementHeightInv = 0, fx = 0, fy = 0, cx = 0, cy = 0;
    std::vector<float> mvScaleFactors; int mnScaleLevels = 0; float mfLogScaleFactor = 0;
    Mat3 R; Vec3 t;
    std::vector<std::vector<std::vector<size_t>>> grid;
    std::vector<std::shared_ptr<S3MP>> mps;
    const std::vector<std::vector<std::vector<size_t>>>& GetGrid() const { return grid; }
    Mat3 GetRotation() const { return R; }
    Vec3 GetTranslation() const { return t; }
    std::vector<std::shared_ptr<S3MP>> GetMapPointMatches() const { return mps; }
};

// view record: n, desc[n*32], angle[n], valid[n] (u8), nodes, per node (id, count, feats[count])
template <class V>
void read_view(FILE* in, V& v, std::vector<KeyPoint>& kps, std::vector<std::shared_ptr<MapPoint>>* mps);

// KeyFrameDatabase mocks: mnId, mBowVec (std::map), covisibility and connections
struct DBKF {
    uint64_t mnId = 0;
    int idx = -1;
    std::map<unsigned int, double> mBowVec;
    std::vector<std::shared_ptr<DBKF>> covis;
    std::set<std::shared_ptr<DBKF>> conn;
    std::vector<std::shared_ptr<DBKF>> GetBestCovisibilityKeyFrames(int n) const {
        return std::vector<std::shared_ptr<DBKF>>(covis.begin(), covis.begin() + std::min<size_t>(n, covis.size()));
    }
    std::set<std::shared_ptr<DBKF>> GetConnectedKeyFrames() const { return conn; }
};
struct DBFrame { uint64_t mnId = 0; std::map<unsigned int, double> mBowVec; };
struct DBVoc { size_t n; size_t size() const { return n; } };

// Frame as PoseOptimization sees it (include/Frame.hpp:52,131,142,145,153,169)
struct PFrame {
    std::vector<KeyPoint> mvKeysUn;
    std::vector<std::shared_ptr<MapPoint>> mvpMapPoints;
    std::vector<float> mvuRight;
    std::vector<bool> mvbOutlier;
    std::vector<float> mvInvLevelSigma2;
    float fx, fy, cx, cy, mbf;
    Mat4 mTcw;
    int set_pose_calls = 0;
    void SetPose(const Mat4& T) { mTcw = T; set_pose_calls++; }
};

template <class T> T rd(FILE* f) { T v; if (fread(&v, sizeof(T), 1, f) != 1) throw std::runtime_error("short read"); return v; }
template <class T> void wr(FILE* f, T v) { fwrite(&v, sizeof(T), 1, f); }

template <class V>
void read_view(FILE* in, V& v, std::vector<KeyPoint>& kps, std::vector<std::shared_ptr<MapPoint>>* mps) {
    v.N = rd<int32_t>(in);
    v.mDescriptors.d.resize(32 * (size_t)v.N);
    if (v.N && fread(v.mDescriptors.d.data(), 1, 32 * (size_t)v.N, in) != 32 * (size_t)v.N) throw std::runtime_error("short read");
    kps.resize(v.N);
    for (int i = 0; i < v.N; ++i) kps[i].angle = rd<float>(in);
    if (mps) mps->resize(v.N);
    for (int i = 0; i < v.N; ++i) {
        const uint8_t ok = rd<uint8_t>(in);  // 0 no map point, 1 good, 2 bad
        if (mps && ok) { auto mp = std::make_shared<MapPoint>(); mp->bad = ok == 2; mp->idx1 = i; (*mps)[i] = mp; }
    }
    const int nn = rd<int32_t>(in);
    for (int k = 0; k < nn; ++k) {
        const uint32_t id = rd<uint32_t>(in), cnt = rd<uint32_t>(in);
        auto& f = v.mFeatVec[id];
        for (uint32_t j = 0; j < cnt; ++j) f.push_back(rd<uint32_t>(in));
    }
}

int main(int argc, char** argv) {
    if (argc != 3) { fprintf(stderr, "usage: facade_test in.bin out.bin\n"); return 2; }
    FILE* in = fopen(argv[1], "rb");
    FILE* out = fopen(argv[2], "wb");
    if (!in || !out) return 2;
    const int mode = rd<int32_t>(in);
    // modes 1-3 compare solvers on their own srand(seed) streams (the opt-in); mode 9 runs on the
    // facade's default, the thread's one reference rand() stream
    if (mode != 9) rsc_orb::reference_rand(false);
    if (mode == 1 || mode == 3) {
        Frame F;
        const int n = rd<int32_t>(in);
        F.fx = rd<float>(in); F.fy = rd<float>(in); F.cx = rd<float>(in); F.cy = rd<float>(in);
        const int nl = rd<int32_t>(in);
        for (int l = 0; l < nl; ++l) F.mvLevelSigma2.push_back(rd<float>(in));
        std::vector<std::shared_ptr<MapPoint>> matches(n);
        F.mvKeysUn.resize(n);
        for (int i = 0; i < n; ++i) {
            const int present = rd<int32_t>(in);
            KeyPoint k; k.pt.x = rd<float>(in); k.pt.y = rd<float>(in); k.octave = rd<int32_t>(in);
            Vec3 X; X.v[0] = rd<float>(in); X.v[1] = rd<float>(in); X.v[2] = rd<float>(in);
            F.mvKeysUn[i] = k;
            if (present) { auto mp = std::make_shared<MapPoint>(); mp->bad = (present == 2); mp->X = X; matches[i] = mp; }
        }
        const uint32_t seed = rd<uint32_t>(in);
        const double prob = rd<double>(in);
        const int mi = rd<int32_t>(in), mx = rd<int32_t>(in), ms = rd<int32_t>(in);
        const float eps = rd<float>(in), th2 = rd<float>(in);
        const int ncalls = rd<int32_t>(in);
        std::unique_ptr<rsc_orb::PnPsolver<Frame, MapPoint>> pnp;
        std::unique_ptr<rsc_orb::MLPnPsolver<Frame, MapPoint>> ml;
        if (mode == 1) {
            pnp.reset(new rsc_orb::PnPsolver<Frame, MapPoint>(F, matches, seed));
            pnp->SetRansacParameters(prob, mi, mx, ms, eps, th2);
        } else {
            ml.reset(new rsc_orb::MLPnPsolver<Frame, MapPoint>(F, matches, seed));
            ml->SetRansacParameters(prob, mi, mx, ms, eps, th2);
        }
        for (int c = 0; c < ncalls; ++c) {
            const int its = rd<int32_t>(in);
            bool nm = false; std::vector<bool> inl; int ni = -1; Mat4 T; std::memset(&T, 0, sizeof(T));
            bool ok = ml ? ml->iterate(its, nm, inl, ni, T)
                         : (its < 0 ? pnp->find(inl, ni, T) : pnp->iterate(its, nm, inl, ni, T));
            wr<int32_t>(out, ok); wr<int32_t>(out, nm); wr<int32_t>(out, ni);
            for (int a = 0; a < 4; ++a) for (int b = 0; b < 4; ++b) wr<float>(out, T.m[a][b]);
            wr<int32_t>(out, (int32_t)inl.size());
            for (bool v : inl) wr<uint8_t>(out, v ? 1 : 0);
        }
    } else if (mode == 9) {
        // Tracking::Relocalization's RANSAC loop (Tracking.cpp:1239-1262) over K candidate Frames with
        // the facade's default (no reference_rand call, no environment variable): every solver draws
        // from the thread's one rand() stream (srand(1), Q3).  Per call: candidate, ok, bNoMore,
        // nInliers, Tcw; ends at the first pose.
        const int K = rd<int32_t>(in);
        const double prob = rd<double>(in);
        const int mi = rd<int32_t>(in), mx = rd<int32_t>(in), ms = rd<int32_t>(in);
        const float eps = rd<float>(in), th2 = rd<float>(in);
        std::vector<Frame> frames(K);
        std::vector<std::vector<std::shared_ptr<MapPoint>>> matches(K);
        std::vector<std::unique_ptr<rsc_orb::PnPsolver<Frame, MapPoint>>> solvers(K);
        for (int k = 0; k < K; ++k) {
            Frame& F = frames[k];
            const int n = rd<int32_t>(in);
            F.fx = rd<float>(in); F.fy = rd<float>(in); F.cx = rd<float>(in); F.cy = rd<float>(in);
            const int nl = rd<int32_t>(in);
            for (int l = 0; l < nl; ++l) F.mvLevelSigma2.push_back(rd<float>(in));
            matches[k].resize(n);
            F.mvKeysUn.resize(n);
            for (int i = 0; i < n; ++i) {
                const int present = rd<int32_t>(in);
                KeyPoint kp; kp.pt.x = rd<float>(in); kp.pt.y = rd<float>(in); kp.octave = rd<int32_t>(in);
                Vec3 X; X.v[0] = rd<float>(in); X.v[1] = rd<float>(in); X.v[2] = rd<float>(in);
                F.mvKeysUn[i] = kp;
                if (present) { auto mp = std::make_shared<MapPoint>(); mp->bad = (present == 2); mp->X = X; matches[k][i] = mp; }
            }
            solvers[k].reset(new rsc_orb::PnPsolver<Frame, MapPoint>(F, matches[k], 1000 + k));
            solvers[k]->SetRansacParameters(prob, mi, mx, ms, eps, th2);
        }
        std::vector<bool> discarded(K, false);
        int nCandidates = K;
        bool bMatch = false;
        while (nCandidates > 0 && !bMatch) {
            for (int i = 0; i < K; ++i) {
                if (discarded[i]) continue;
                bool nm = false; std::vector<bool> inl; int ni = -1; Mat4 T; std::memset(&T, 0, sizeof(T));
                const bool ok = solvers[i]->iterate(5, nm, inl, ni, T);
                wr<int32_t>(out, i); wr<int32_t>(out, ok); wr<int32_t>(out, nm); wr<int32_t>(out, ni);
                for (int a = 0; a < 4; ++a) for (int b = 0; b < 4; ++b) wr<float>(out, T.m[a][b]);
                if (nm) { discarded[i] = true; nCandidates--; }
                if (ok) { bMatch = true; break; }
            }
        }
        wr<int32_t>(out, -1);
        int64_t pos = -1;
        rsc_stream_position(rsc_orb::thread_stream(), &pos);
        wr<int64_t>(out, pos);
    } else if (mode == 4) {
        // Optimizer::PoseOptimization on a mock Frame: n slots, fx..cy, mbf, Tcw, levels of
        // mvInvLevelSigma2, per slot (present, u, v, octave, X, uR)
        PFrame F;
        const int n = rd<int32_t>(in);
        F.fx = rd<float>(in); F.fy = rd<float>(in); F.cx = rd<float>(in); F.cy = rd<float>(in);
        F.mbf = rd<float>(in);
        for (int r = 0; r < 4; ++r) for (int c = 0; c < 4; ++c) F.mTcw.m[r][c] = rd<float>(in);
        const int nl = rd<int32_t>(in);
        for (int l = 0; l < nl; ++l) F.mvInvLevelSigma2.push_back(rd<float>(in));
        F.mvKeysUn.resize(n);
        F.mvpMapPoints.resize(n);
        F.mvuRight.resize(n);
        F.mvbOutlier.assign(n, true);
        for (int i = 0; i < n; ++i) {
            const int present = rd<int32_t>(in);
            KeyPoint k; k.pt.x = rd<float>(in); k.pt.y = rd<float>(in); k.octave = rd<int32_t>(in);
            Vec3 X; X.v[0] = rd<float>(in); X.v[1] = rd<float>(in); X.v[2] = rd<float>(in);
            F.mvuRight[i] = rd<float>(in);
            F.mvKeysUn[i] = k;
            if (present) { auto mp = std::make_shared<MapPoint>(); mp->X = X; F.mvpMapPoints[i] = mp; }
        }
        const int nGood = rsc_orb::PoseOptimization(&F);
        wr<int32_t>(out, nGood);
        wr<int32_t>(out, F.set_pose_calls);
        for (int a = 0; a < 4; ++a) for (int b = 0; b < 4; ++b) wr<float>(out, F.mTcw.m[a][b]);
        for (int i = 0; i < n; ++i) wr<uint8_t>(out, F.mvbOutlier[i] ? 1 : 0);
    } else if (mode == 5) {
        // ORBmatcher::SearchByBoW through rsc_orb::ORBmatcher: frame overload (pKF = views[c], F =
        // shared) or KeyFrame overload (pKF1 = shared, pKF2 = views[c]); writes nmatches and, per
        // slot of the result vector, the matched MapPoint's feature index in its KeyFrame or -1
        const int frame_overload = rd<int32_t>(in);
        const float ratio = rd<float>(in);
        const int check = rd<int32_t>(in);
        const int C = rd<int32_t>(in);
        rsc_orb::ORBmatcher matcher(ratio, check != 0);
        if (frame_overload) {
            BowFrame F;
            read_view(in, F, F.mvKeys, nullptr);
            std::vector<std::shared_ptr<BowKF>> kfs(C);
            for (auto& k : kfs) { k = std::make_shared<BowKF>(); read_view(in, *k, k->mvKeysUn, &k->mps); }
            for (int c = 0; c < C; ++c) {  // the reference's per-candidate calls (Tracking.cpp:1214)
                std::vector<std::shared_ptr<MapPoint>> m;
                const int nm = matcher.SearchByBoW(kfs[c], F, m);
                wr<int32_t>(out, nm);
                wr<int32_t>(out, (int32_t)m.size());
                for (auto& mp : m) wr<int32_t>(out, mp ? mp->idx1 : -1);
            }
            std::vector<std::vector<std::shared_ptr<MapPoint>>> mm;  // batched form, same results
            const std::vector<int> nms = matcher.SearchByBoWMany(kfs, F, mm);
            for (int c = 0; c < C; ++c) {
                wr<int32_t>(out, nms[c]);
                for (auto& mp : mm[c]) wr<int32_t>(out, mp ? mp->idx1 : -1);
            }
        } else {
            auto K1 = std::make_shared<BowKF>();
            read_view(in, *K1, K1->mvKeysUn, &K1->mps);
            std::vector<std::shared_ptr<BowKF>> kfs(C);
            for (auto& k : kfs) { k = std::make_shared<BowKF>(); read_view(in, *k, k->mvKeysUn, &k->mps); }
            for (int c = 0; c < C; ++c) {  // LoopClosing.cpp:251
                std::vector<std::shared_ptr<MapPoint>> m;
                const int nm = matcher.SearchByBoW(K1, kfs[c], m);
                wr<int32_t>(out, nm);
                wr<int32_t>(out, (int32_t)m.size());
                for (auto& mp : m) wr<int32_t>(out, mp ? mp->idx1 : -1);
            }
            std::vector<std::vector<std::shared_ptr<MapPoint>>> mm;
            const std::vector<int> nms = matcher.SearchByBoWMany(K1, kfs, mm);
            for (int c = 0; c < C; ++c) {
                wr<int32_t>(out, nms[c]);
                for (auto& mp : mm[c]) wr<int32_t>(out, mp ? mp->idx1 : -1);
            }
        }
    } else if (mode == 6) {
        // KeyFrameDatabase through rsc_orb::KeyFrameDatabase: a table of KeyFrames (BowVector,
        // covisibility), then add / erase / clear / relocalization / loop operations; writes each
        // query's candidates as KeyFrame table indices
        auto read_bow = [&](std::map<unsigned int, double>& b) {
            const int n = rd<int32_t>(in);
            std::vector<uint32_t> ids(n);
            for (auto& x : ids) x = rd<uint32_t>(in);
            for (int i = 0; i < n; ++i) b[ids[i]] = rd<double>(in);
        };
        auto voc = std::make_shared<DBVoc>(DBVoc{rd<uint32_t>(in)});
        const int K = rd<int32_t>(in);
        std::vector<std::shared_ptr<DBKF>> kfs(K);
        for (int k = 0; k < K; ++k) { kfs[k] = std::make_shared<DBKF>(); kfs[k]->idx = k; kfs[k]->mnId = 100000 + k; }
        for (int k = 0; k < K; ++k) {
            read_bow(kfs[k]->mBowVec);
            const int nc = rd<int32_t>(in);
            for (int j = 0; j < nc; ++j) kfs[k]->covis.push_back(kfs[rd<int32_t>(in)]);
        }
        rsc_orb::KeyFrameDatabase<std::shared_ptr<DBKF>> db(voc, K + 64);
        const int nops = rd<int32_t>(in);
        for (int o = 0; o < nops; ++o) {
            const int kind = rd<int32_t>(in);
            std::vector<std::shared_ptr<DBKF>> cands;
            if (kind == 0) { db.add(kfs[rd<int32_t>(in)]); continue; }
            if (kind == 1) { db.erase(kfs[rd<int32_t>(in)]); continue; }
            if (kind == 2) { db.clear(); continue; }
            if (kind == 4) {
                DBFrame F;
                F.mnId = rd<uint64_t>(in);
                read_bow(F.mBowVec);
                cands = db.DetectRelocalizationCandidates(&F);
            } else {
                auto q = std::make_shared<DBKF>();
                q->mnId = rd<uint64_t>(in);
                read_bow(q->mBowVec);
                const int nc = rd<int32_t>(in);
                for (int j = 0; j < nc; ++j) q->conn.insert(kfs[rd<int32_t>(in)]);
                const float ms = rd<float>(in);
                cands = db.DetectLoopCandidates(q, ms);
            }
            wr<int32_t>(out, (int32_t)cands.size());
            for (auto& c : cands) wr<int32_t>(out, c->idx);
        }
    } else if (mode == 7) {
        // ORBmatcher::SearchBySim3 through the facade: two KeyFrames (keypoints, octaves,
        // descriptors, CSR grid, bounds, intrinsics, scale pyramid, pose, MapPoints), R12, t12, th,
        // matched12 (KF2 index / -1 NULL / -2 a MapPoint not in KF2); writes nfound and vpMatches12
        // after the call as KF2 indices (-1 NULL, -2 the foreign MapPoint)
        std::shared_ptr<S3KF> kf[2] = {std::make_shared<S3KF>(), std::make_shared<S3KF>()};
        for (auto& k : kf) {
            const int n = rd<int32_t>(in);
            k->N = n;
            k->mvKeysUn.resize(n);
            for (int i = 0; i < n; ++i) { k->mvKeysUn[i].pt.x = rd<float>(in); k->mvKeysUn[i].pt.y = rd<float>(in); }
            for (int i = 0; i < n; ++i) k->mvKeysUn[i].octave = rd<int32_t>(in);
            k->mDescriptors.d.resize(32 * (size_t)n);
            if (n && fread(k->mDescriptors.d.data(), 1, 32 * (size_t)n, in) != 32 * (size_t)n) throw std::runtime_error("short read");
            std::vector<int32_t> begin(64 * 48 + 1);
            for (auto& b : begin) b = rd<int32_t>(in);
            k->grid.assign(64, std::vector<std::vector<size_t>>(48));
            for (int c = 0; c < 64 * 48; ++c)
                for (int j = begin[c]; j < begin[c + 1]; ++j) k->grid[c / 48][c % 48].push_back((size_t)rd<int32_t>(in));
            k->mnMinX = rd<int32_t>(in); k->mnMaxX = rd<int32_t>(in); k->mnMinY = rd<int32_t>(in); k->mnMaxY = rd<int32_t>(in);
            k->mfGridElementWidthInv = rd<float>(in); k->mfGridElementHeightInv = rd<float>(in);
            k->fx = rd<float>(in); k->fy = rd<float>(in); k->cx = rd<float>(in); k->cy = rd<float>(in);
            k->mnScaleLevels = rd<int32_t>(in);
            for (int l = 0; l < k->mnScaleLevels; ++l) k->mvScaleFactors.push_back(rd<float>(in));
            k->mfLogScaleFactor = rd<float>(in);
            for (int r = 0; r < 3; ++r) for (int c = 0; c < 3; ++c) k->R.m[r][c] = rd<float>(in);
            for (int r = 0; r < 3; ++r) k->t.v[r] = rd<float>(in);
            k->mps.resize(n);
            for (int i = 0; i < n; ++i) {
                const int st = rd<uint8_t>(in);
                auto mp = std::make_shared<S3MP>();
                for (int c = 0; c < 3; ++c) mp->X.v[c] = rd<float>(in);
                mp->dmax = rd<float>(in); mp->dmin = rd<float>(in);
                mp->d.d.resize(32);
                if (fread(mp->d.d.data(), 1, 32, in) != 32) throw std::runtime_error("short read");
                mp->bad = st == 2; mp->home = k.get(); mp->idx = i;
                if (st) k->mps[i] = mp;
            }
        }
        Mat3 R12; Vec3 t12;
        for (int r = 0; r < 3; ++r) for (int c = 0; c < 3; ++c) R12.m[r][c] = rd<float>(in);
        for (int r = 0; r < 3; ++r) t12.v[r] = rd<float>(in);
        const float th = rd<float>(in);
        auto foreign = std::make_shared<S3MP>();
        std::vector<std::shared_ptr<S3MP>> m12(kf[0]->N);
        for (int i = 0; i < kf[0]->N; ++i) {
            const int v = rd<int32_t>(in);
            if (v >= 0) m12[i] = kf[1]->mps[v];
            else if (v == -2) m12[i] = foreign;
        }
        rsc_orb::ORBmatcher matcher;
        const int nf = matcher.SearchBySim3(kf[0], kf[1], m12, R12, t12, th);
        wr<int32_t>(out, nf);
        for (auto& mp : m12) wr<int32_t>(out, !mp ? -1 : (mp == foreign ? -2 : mp->idx));
    } else if (mode == 8) {
        // Optimizer::OptimizeSim3 through the facade: n1 slots of KF1, n2 of KF2, per KF pose, K,
        // inverse level sigmas; per KF2 slot (u, v, octave); per KF1 slot (u, v, octave, kind, X1,
        // X2, i2) with kind 0 = vpMatches1 NULL, 1 = pMP1 NULL, 2 = pMP1 bad, 3 = pMP2 bad, 4 = i2 < 0,
        // 5 = a correspondence; then S[8], th2.  Writes nIn, S after the call, and per slot whether
        // vpMatches1[i] is still set.
        auto kf1 = std::make_shared<KeyFrame>(), kf2 = std::make_shared<KeyFrame>();
        const int n1 = rd<int32_t>(in), n2 = rd<int32_t>(in);
        for (auto* kf : {kf1.get(), kf2.get()}) {
            for (int r = 0; r < 3; ++r) for (int c = 0; c < 3; ++c) kf->R.m[r][c] = rd<float>(in);
            for (int r = 0; r < 3; ++r) kf->t.v[r] = rd<float>(in);
            float K[4]; for (float& k : K) k = rd<float>(in);
            std::memset(&kf->mK, 0, sizeof(Mat3));
            kf->mK.m[0][0] = K[0]; kf->mK.m[1][1] = K[1]; kf->mK.m[0][2] = K[2]; kf->mK.m[1][2] = K[3]; kf->mK.m[2][2] = 1;
            const int nl = rd<int32_t>(in);
            for (int l = 0; l < nl; ++l) kf->mvInvLevelSigma2.push_back(rd<float>(in));
        }
        kf1->mvKeysUn.resize(n1); kf1->mps.resize(n1);
        kf2->mvKeysUn.resize(n2); kf2->mps.resize(n2);
        for (int j = 0; j < n2; ++j) { kf2->mvKeysUn[j].pt.x = rd<float>(in); kf2->mvKeysUn[j].pt.y = rd<float>(in); kf2->mvKeysUn[j].octave = rd<int32_t>(in); }
        std::vector<std::shared_ptr<MapPoint>> m1(n1);
        for (int i = 0; i < n1; ++i) {
            kf1->mvKeysUn[i].pt.x = rd<float>(in); kf1->mvKeysUn[i].pt.y = rd<float>(in); kf1->mvKeysUn[i].octave = rd<int32_t>(in);
            const int kind = rd<int32_t>(in);
            Vec3 a, b; for (int r = 0; r < 3; ++r) a.v[r] = rd<float>(in);
            for (int r = 0; r < 3; ++r) b.v[r] = rd<float>(in);
            const int i2 = rd<int32_t>(in);
            if (kind == 0) continue;
            if (kind != 1) {
                auto mp1 = std::make_shared<MapPoint>(); mp1->X = a; mp1->bad = kind == 2; mp1->kf1 = kf1.get(); mp1->idx1 = i;
                kf1->mps[i] = mp1;
            }
            auto mp2 = std::make_shared<MapPoint>(); mp2->X = b; mp2->bad = kind == 3; mp2->kf1 = kf1.get();
            mp2->idx1 = -1; mp2->idx2 = kind == 4 ? -1 : i2;
            m1[i] = mp2;
        }
        MockSim3 S;
        for (int k = 0; k < 4; ++k) S.q.c.v[k] = rd<double>(in);
        for (int k = 0; k < 3; ++k) S.tr.v[k] = rd<double>(in);
        S.s = rd<double>(in);
        const float th2 = rd<float>(in);
        const int nIn = rsc_orb::OptimizeSim3(kf1, kf2, m1, S, th2);
        wr<int32_t>(out, nIn);
        for (int k = 0; k < 4; ++k) wr<double>(out, S.q.c.v[k]);
        for (int k = 0; k < 3; ++k) wr<double>(out, S.tr.v[k]);
        wr<double>(out, S.s);
        for (int i = 0; i < n1; ++i) wr<uint8_t>(out, m1[i] ? 1 : 0);
    } else if (mode == 2) {
        auto kf1 = std::make_shared<KeyFrame>(), kf2 = std::make_shared<KeyFrame>();
        const int n1 = rd<int32_t>(in);
        for (auto* kf : {kf1.get(), kf2.get()}) {
            for (int r = 0; r < 3; ++r) for (int c = 0; c < 3; ++c) kf->R.m[r][c] = rd<float>(in);
            for (int r = 0; r < 3; ++r) kf->t.v[r] = rd<float>(in);
            float K[4]; for (float& k : K) k = rd<float>(in);
            std::memset(&kf->mK, 0, sizeof(Mat3));
            kf->mK.m[0][0] = K[0]; kf->mK.m[1][1] = K[1]; kf->mK.m[0][2] = K[2]; kf->mK.m[1][2] = K[3]; kf->mK.m[2][2] = 1;
            const int nl = rd<int32_t>(in);
            for (int l = 0; l < nl; ++l) kf->mvLevelSigma2.push_back(rd<float>(in));
            kf->mvKeysUn.resize(n1);
            kf->mps.resize(n1);
        }
        std::vector<std::shared_ptr<MapPoint>> matched(n1);
        for (int i = 0; i < n1; ++i) {
            const int flags = rd<int32_t>(in);  // bit0 matched, bit1 mp1, bit2 bad1, bit3 bad2, bit4 idx1 invalid, bit5 idx2 invalid
            Vec3 a, b; for (int r = 0; r < 3; ++r) a.v[r] = rd<float>(in);
            for (int r = 0; r < 3; ++r) b.v[r] = rd<float>(in);
            const int o1 = rd<int32_t>(in), o2 = rd<int32_t>(in);
            kf1->mvKeysUn[i].octave = o1;
            kf2->mvKeysUn[i].octave = o2;
            if (flags & 2) {
                auto mp1 = std::make_shared<MapPoint>(); mp1->X = a; mp1->bad = flags & 4; mp1->kf1 = kf1.get();
                mp1->idx1 = (flags & 16) ? -1 : i; mp1->idx2 = -1; kf1->mps[i] = mp1;
            }
            if (flags & 1) {
                auto mp2 = std::make_shared<MapPoint>(); mp2->X = b; mp2->bad = flags & 8; mp2->kf1 = kf1.get();
                mp2->idx1 = -1; mp2->idx2 = (flags & 32) ? -1 : i; matched[i] = mp2;
            }
        }
        const uint32_t seed = rd<uint32_t>(in);
        const double prob = rd<double>(in);
        const int mi = rd<int32_t>(in), mx = rd<int32_t>(in);
        const int ncalls = rd<int32_t>(in);
        // LoopClosing::ComputeSim3's own expressions (LoopClosing.cpp:260-261,286,307-308): the
        // solvers live behind pointers and the getters are called without template arguments.
        std::vector<std::shared_ptr<rsc_orb::Sim3Solver<KeyFrame, MapPoint>>> vpSim3Solvers(1);
        vpSim3Solvers[0] = std::make_shared<rsc_orb::Sim3Solver<KeyFrame, MapPoint>>(kf1, kf2, matched, seed);
        auto& solver = *vpSim3Solvers[0];
        solver.SetRansacParameters(prob, mi, mx);
        for (int c = 0; c < ncalls; ++c) {
            const int its = rd<int32_t>(in);
            bool nm = false; std::vector<bool> inl; int ni = -1;
            bool ok = its < 0 ? solver.find(inl, ni) : vpSim3Solvers[0]->iterate(its, nm, inl, ni);
            Mat3 R = vpSim3Solvers[0]->GetEstimatedRotation();
            Vec3 t = vpSim3Solvers[0]->GetEstimatedTranslation();
            {   // the explicit-type form gives the same values
                Mat3 R2 = solver.GetEstimatedRotation<Mat3>();
                Vec3 t2 = solver.GetEstimatedTranslation<Vec3>();
                if (std::memcmp(&R2, &R, sizeof(R)) || std::memcmp(&t2, &t, sizeof(t))) return 3;
            }
            wr<int32_t>(out, ok); wr<int32_t>(out, nm); wr<int32_t>(out, ni);
            for (int a = 0; a < 3; ++a) for (int b = 0; b < 3; ++b) wr<float>(out, R.m[a][b]);
            for (int a = 0; a < 3; ++a) wr<float>(out, t.v[a]);
            wr<int32_t>(out, (int32_t)inl.size());
            for (bool v : inl) wr<uint8_t>(out, v ? 1 : 0);
        }
    }
    fclose(in);
    fclose(out);
    return 0;
}
