// TEST INFRASTRUCTURE (CPU model, tests/test_wide_walk.py): record visits and child box tests per path segment of a
// K-wide tree collapsed from the reference's binary tree by the surface-area-optimal cut
// (pt_wide.cpp's dynamic programme with K members), walked in preorder with children culled
// at the t of the record visit (the wide walk's rule), K = 2 / 4 / 8; exact boxes.
#include "../../oracle/pt_oracle.cpp"
#include <cstdio>
#include <fstream>
#include <functional>
static std::vector<float> loadf(const char* p) {
    std::ifstream f(p, std::ios::binary); f.seekg(0, std::ios::end); size_t n = f.tellg() / 4; f.seekg(0);
    std::vector<float> v(n); f.read((char*)v.data(), n * 4); return v;
}
namespace {
const Scene* g_sc;
std::vector<int> L, R;
double area(int i) { const float* b = g_sc->nodes + 12 * i; double x = b[4] - b[0], y = b[5] - b[1], z = b[6] - b[2];
    return 2 * (x * y + y * z + z * x); }
struct Wide { std::vector<std::vector<int>> kids; std::vector<int> rec_of; };   // per binary node that is a record
Wide build(int K) {
    int n = g_sc->nn; std::vector<std::vector<double>> F(n, std::vector<double>(K + 1, 0));
    std::vector<std::vector<int>> sp(n, std::vector<int>(K + 1, 0));
    std::vector<int> order, st{0};
    while (!st.empty()) { int x = st.back(); st.pop_back(); order.push_back(x); if (L[x] >= 0) { st.push_back(L[x]); st.push_back(R[x]); } }
    for (auto it = order.rbegin(); it != order.rend(); ++it) {
        int y = *it; if (L[y] < 0) continue; int l = L[y], r = R[y];
        double best = 1e300; for (int k1 = 1; k1 < K; k1++) best = std::min(best, F[l][k1] + F[r][K - k1]);
        F[y][1] = (area(y) + 1e-30) + best;
        for (int k = 2; k <= K; k++) { F[y][k] = F[y][k - 1]; sp[y][k] = sp[y][k - 1];
            for (int k1 = 1; k1 < k; k1++) { double c = F[l][k1] + F[r][k - k1]; if (c < F[y][k]) { F[y][k] = c; sp[y][k] = k1; } } }
    }
    std::function<void(int, int, std::vector<int>&)> expand = [&](int y, int k, std::vector<int>& f) {
        int k1 = L[y] < 0 ? 0 : sp[y][k]; if (k1 == 0) { f.push_back(y); return; }
        expand(L[y], k1, f); expand(R[y], k - k1, f); };
    Wide w; w.rec_of.assign(n, -1);
    std::vector<int> q{0};
    while (!q.empty()) {
        int x = q.back(); q.pop_back(); if (w.rec_of[x] >= 0) continue;
        std::vector<int> f;
        if (L[x] < 0) f.push_back(x);
        else { int l = L[x], r = R[x], bk = 1; double best = 1e300;
            for (int k1 = 1; k1 < K; k1++) if (F[l][k1] + F[r][K - k1] < best) { best = F[l][k1] + F[r][K - k1]; bk = k1; }
            expand(l, bk, f); expand(r, K - bk, f); }
        w.rec_of[x] = (int)w.kids.size(); w.kids.push_back(f);
        for (int c : f) if (L[c] >= 0) q.push_back(c);
    }
    return w;
}
struct St { double seg = 0, visits = 0, tests = 0, leaves = 0, mism = 0; };
void walk(const Wide& w, int rec, V3 o, V3 d, float& t, int& prim, St& s) {
    s.visits++;
    const auto& f = w.kids[rec];
    bool hit[64]; int m = (int)f.size();
    for (int j = 0; j < m; j++) { s.tests++; hit[j] = bvh_intersect(g_sc->nodes + 12 * f[j], o, d, t); }
    V3 rn, rn2;
    for (int j = 0; j < m; j++) {
        if (!hit[j]) continue;
        int c = f[j];
        if (L[c] < 0) {
            // the reference re-tests the leaf's box at the current t before its triangles count
            s.leaves++;
            const float* b = g_sc->nodes + 12 * c;
            if (!bvh_intersect(b, o, d, t)) continue;
            int t0 = (int)b[8], t1 = (int)b[9];
            float h1 = hit_triangle(o, d, g_sc->tris + 16 * t0, rn), h2 = hit_triangle(o, d, g_sc->tris + 16 * t1, rn2);
            if (h1 > 0.0001f && h1 < t && (h1 < h2 || h2 < 0.0001f)) { t = h1; prim = t0; }
            else if (h2 > 0.0001f && h2 < t) { t = h2; prim = t1; }
        } else walk(w, w.rec_of[c], o, d, t, prim, s);
    }
}
void ref_hit(V3 o, V3 d, float& t, int& prim) {
    const Scene& sc = *g_sc; t = std::numeric_limits<float>::infinity(); prim = -1;
    for (int si = 0; si < sc.ns; si++) { float ht = hit_sphere(o, d, sc.spheres + 8 * si); if (ht > 0.0001f && ht < t) { t = ht; prim = -2 - si; } }
    V3 rn, rn2;
    for (int bi = 0; bi > -1;) {
        const float* b = sc.nodes + 12 * bi; bool hb = bvh_intersect(b, o, d, t); int next = hb ? (int)b[10] : (int)b[11];
        if (hb && (b[8] > -1.0f)) { int t0 = (int)b[8], t1 = (int)b[9];
            float h1 = hit_triangle(o, d, sc.tris + 16 * t0, rn), h2 = hit_triangle(o, d, sc.tris + 16 * t1, rn2);
            if (h1 > 0.0001f && h1 < t && (h1 < h2 || h2 < 0.0001f)) { t = h1; prim = t0; } else if (h2 > 0.0001f && h2 < t) { t = h2; prim = t1; } }
        bi = next;
    }
}
}  // namespace
int main(int argc, char** argv) {
    if (argc < 3) { fprintf(stderr, "usage: widek_sim scene.bin stride\n"); return 2; }
    int stride = atoi(argv[2]);
    std::vector<float> all = loadf(argv[1]);
    int cnt[4];
    std::memcpy(cnt, all.data(), 16);
    size_t off = 4;
    auto take = [&](size_t n) { std::vector<float> v(all.begin() + off, all.begin() + off + n); off += n; return v; };
    auto tris = take((size_t)cnt[0] * 16), nodes = take((size_t)cnt[1] * 12), mats = take((size_t)cnt[2] * 16),
         sph = take((size_t)cnt[3] * 8), cam = take(12);
    Scene sc{tris.data(), (int)tris.size() / 16, nodes.data(), (int)nodes.size() / 12, mats.data(), (int)mats.size() / 16, sph.data(), (int)sph.size() / 8};
    g_sc = &sc;
    L.assign(sc.nn, -1); R.assign(sc.nn, -1);
    for (int i = 0; i < sc.nn; i++) { const float* b = sc.nodes + 12 * i; if (b[8] > -1.0f) continue; L[i] = (int)b[10]; R[i] = L[i] + 1; }
    int Ks[3] = {2, 4, 8}; Wide W[3]; St S[3];
    for (int q = 0; q < 3; q++) W[q] = build(Ks[q]);
    const int Wd = 1920, Hd = 1080; Camera c = make_camera(cam.data(), Wd, Hd);
    for (int yy = 0; yy < Hd; yy += stride) for (int xx = 0; xx < Wd; xx += stride) {
        uint32_t pix = (uint32_t)yy * 831266u + (uint32_t)xx * 923766u; uint32_t state = pix + 719393u;
        float ax = random01(state), ay = random01(state);
        float u = ((float)xx + ax) / (float)Wd - 0.5f, v = ((float)yy + ay) / (float)Hd - 0.5f;
        V3 d = normalize(add(add(c.fwd, muls(c.right, u)), muls(c.up, v))), o = c.pos, col = v3(1, 1, 1);
        for (int i = 0; i <= 8; i++) {
            float t0; int p0; ref_hit(o, d, t0, p0);
            for (int q = 0; q < 3; q++) {
                float t = std::numeric_limits<float>::infinity(); int prim = -1;
                for (int si = 0; si < sc.ns; si++) { float ht = hit_sphere(o, d, sc.spheres + 8 * si); if (ht > 0.0001f && ht < t) { t = ht; prim = -2 - si; } }
                S[q].seg++; walk(W[q], 0, o, d, t, prim, S[q]);
                if (std::memcmp(&t, &t0, 4) != 0 || prim != p0) S[q].mism++;
            }
            if (p0 == -1) break;
            V3 hp = add(o, muls(d, t0)), nrm; int mat;
            if (p0 <= -2) { nrm = normalize(sub(hp, ld3(sc.spheres))); mat = (int)sc.spheres[4]; }
            else { V3 rn; hit_triangle(o, d, sc.tris + 16 * p0, rn); nrm = rn; mat = (int)sc.tris[16 * p0 + 12]; }
            if (dot(nrm, d) > 0.0f) nrm = muls(nrm, -1.0f);
            if (!(length(col) > 0.01f)) break;
            o = hp; V3 diff = normalize(add(nrm, random_unit_vector(state))); float k = 2.0f * dot(nrm, d);
            V3 spec = normalize(sub(d, muls(nrm, k))); const float* m = sc.mats + 16 * mat;
            float is_spec = m[14] > random01(state) ? 1.0f : 0.0f; d = mixv(diff, spec, m[13] * is_spec);
            col = mul(col, mixv(ld3(m), ld3(m + 8), is_spec));
        }
    }
    printf("{\"segments\": %.0f", S[0].seg);
    for (int q = 0; q < 3; q++)
        printf(", \"K%d\": {\"records\": %zu, \"visits\": %.4f, \"child_tests\": %.4f, \"leaves\": %.4f, \"mismatches\": %.0f}", Ks[q],
               W[q].kids.size(), S[q].visits / S[q].seg, S[q].tests / S[q].seg, S[q].leaves / S[q].seg, S[q].mism);
    printf("}\n");
}
