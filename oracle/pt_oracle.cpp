// =====================================================================================
//  oracle/pt_oracle.cpp  --  TEST INFRASTRUCTURE ONLY.  NOT PART OF THE PRODUCT.
//
//  A plain C++ CPU restatement of the reference hot path (danielbrathwaite/OpenGL-Path-
//  Tracing, LearnOpenGL/computeShader.c) and of the host code that feeds it (OBJ/MTL
//  loader, SAH BVH builder, setupBuffers scene assembly).  It is written from the
//  reference files read as text; no reference source is compiled, linked or copied.
//
//  Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may load this
//  library, and only as the checker / the timed CPU baseline.  The product
//  (opengl-path-tracing_amd/) never includes, links or calls anything in oracle/.
//
//  Parity status: the reference has no golden vectors and cannot be executed here (no GL
//  context; executing reference code was refused).  This oracle is
//  therefore pinned by (1) known-answer tests derived by hand from the spec, (2) an
//  independent numpy-float32 twin (oracle/numpy_twin.py) that must agree bit-for-bit,
//  and (3) the reference's own data files (scene_data/*.txt) for the loader/BVH.
//  Parity against any real GL driver is UNPINNED (GLSL transcendental precision is
//  implementation-defined).  See DESIGN.md §3.
//
//  Arithmetic pinning: every float expression below is evaluated in
//  IEEE binary32, round-to-nearest, left to right, no FMA contraction (-ffp-contract=off),
//  correctly rounded '/' and sqrtf.  dot(a,b) = (a.x*b.x + a.y*b.y) + a.z*b.z;
//  cross per the GLSL spec; normalize(v) = v * (1/sqrt(dot(v,v))); mix(x,y,a) =
//  x*(1-a) + y*a; log / cos = the build's pinned polynomials (o_logf / o_cosf below).
// =====================================================================================
#include <algorithm>
#include <atomic>
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <fstream>
#include <limits>
#include <sstream>
#include <string>
#include <thread>
#include <unordered_map>
#include <vector>

#if defined(__FP_FAST_FMAF) && !defined(PT_ORACLE_ALLOW_FMA)
// fine: contraction is what matters and the Makefile passes -ffp-contract=off
#endif

namespace {

// ------------------------------------------------------------------ scalar helpers
inline uint32_t f2u(float f) { uint32_t u; std::memcpy(&u, &f, 4); return u; }
inline float u2f(uint32_t u) { float f; std::memcpy(&f, &u, 4); return f; }

// The Box-Muller log and cos (computeShader.c:115-120).  GLSL leaves their precision to the
// GL driver; the build pins one choice (opengl-path-tracing_amd/csrc/pt_math.h logf_pinned /
// cosf_pinned), restated here from its definition:
//   log x, x in {0} U [2^-32, 1]: split x = 2^k z at the exponent boundary 0x3f330000
//     (z in [0.699, 1.398)); f = z - 1; log = f + f^2 P(f) (Horner in fma, 8 coefficients)
//     + k ln2_lo, then + k ln2_hi; log 0 = -inf.
//   cos t, t in [0, 2 pi]: q = rint(t * 2/pi); r = t - q pi/2 (pi/2 in two parts, by fma);
//     quadrant q mod 4 picks cos r (1 + r^2 C(r^2)) or sin r (r + r^3 S(r^2)); the sign is
//     negative in quadrants 1 and 2.
// std::fma is the correctly rounded fused multiply-add (the GPU's v_fma_f32).
const float kLogP[8] = {0x1.87c9c0p-4f, -0x1.2bf636p-3f, 0x1.2f3194p-3f, -0x1.52694ep-3f,
                        0x1.98eb62p-3f, -0x1.000924p-2f, 0x1.5556ccp-2f, -0x1.fffff0p-2f};
float o_logf(float x) {
    if (x == 0.0f) return -std::numeric_limits<float>::infinity();
    const uint32_t ix = f2u(x);
    const uint32_t split = ix - 0x3f330000u;
    const int k = (int32_t)split >> 23;                     // arithmetic shift: k in [-32, 0]
    const float z = u2f(ix - (split & 0xff800000u));
    const float f = z - 1.0f;
    float P = kLogP[0];
    for (int i = 1; i < 8; i++) P = std::fma(f, P, kLogP[i]);
    const float kf = (float)k;
    float y = std::fma(f * f, P, f);
    y = std::fma(kf, 0x1.2fefa2p-17f, y);                  // k ln2_lo
    return std::fma(kf, 0x1.62e300p-1f, y);                // + k ln2_hi
}

float o_cosf(float t) {
    const float q = std::nearbyint(t * 0x1.45f306p-1f);    // ties to even (default mode)
    float r = std::fma(-q, 0x1.921fb6p+0f, t);
    r = std::fma(-q, -0x1.777a5cp-25f, r);
    const float r2 = r * r;
    float cpoly = std::fma(r2, -0x1.64756cp-10f, 0x1.553f94p-5f);
    cpoly = std::fma(r2, cpoly, -0x1.ffffbap-2f);
    const float c = std::fma(r2, cpoly, 1.0f);
    float spoly = std::fma(r2, -0x1.98da64p-13f, 0x1.1105b4p-7f);
    spoly = std::fma(r2, spoly, -0x1.555540p-3f);
    const float sn = std::fma(r * r2, spoly, r);
    const int quadrant = ((int)q) & 3;
    const float v = (quadrant & 1) ? sn : c;
    return (quadrant == 1 || quadrant == 2) ? -v : v;
}

struct V3 { float x, y, z; };
inline V3 v3(float x, float y, float z) { return {x, y, z}; }
inline V3 add(V3 a, V3 b) { return {a.x + b.x, a.y + b.y, a.z + b.z}; }
inline V3 sub(V3 a, V3 b) { return {a.x - b.x, a.y - b.y, a.z - b.z}; }
inline V3 mul(V3 a, V3 b) { return {a.x * b.x, a.y * b.y, a.z * b.z}; }
inline V3 muls(V3 a, float s) { return {a.x * s, a.y * s, a.z * s}; }
inline V3 divs(V3 a, float s) { return {a.x / s, a.y / s, a.z / s}; }
inline float dot(V3 a, V3 b) { return (a.x * b.x + a.y * b.y) + a.z * b.z; }
inline V3 cross(V3 a, V3 b) {
    return {a.y * b.z - b.y * a.z, a.z * b.x - b.z * a.x, a.x * b.y - b.x * a.y};
}
inline float length(V3 a) { return std::sqrt(dot(a, a)); }
inline V3 normalize(V3 a) { float r = 1.0f / std::sqrt(dot(a, a)); return muls(a, r); }
inline V3 mixv(V3 x, V3 y, float a) {
    float oma = 1.0f - a;
    return {x.x * oma + y.x * a, x.y * oma + y.y * a, x.z * oma + y.z * a};
}
inline V3 ld3(const float* p) { return {p[0], p[1], p[2]}; }

// ---------------------------------------------------------- RNG (computeShader.c:87-129)
inline uint32_t next_random(uint32_t& s) {
    s = s * 747796405u + 2891336453u;
    uint32_t r = ((s >> ((s >> 28) + 4)) ^ s) * 277803737u;
    r = (r >> 22) ^ r;
    return r;
}
// NextRandom(state) / 4294967295.0 : the float literal rounds to 2^32, uint -> float rounds.
inline float random01(uint32_t& s) { return (float)next_random(s) * (1.0f / 4294967296.0f); }
inline float random_normal(uint32_t& s) {                      // :115-120
    float theta = (2.0f * 3.1415926f) * random01(s);
    float rho = std::sqrt(-2.0f * o_logf(random01(s)));
    return rho * o_cosf(theta);
}
inline V3 random_unit_vector(uint32_t& s) {                   // :122-129, x then y then z
    float x = random_normal(s);
    float y = random_normal(s);
    float z = random_normal(s);
    return normalize(v3(x, y, z));
}
inline V3 environment_light(V3 d) {                            // :131-140
    V3 dir = normalize(d);
    float t = 0.5f * (dir.z + 1.0f);
    float omt = 1.0f - t;
    return {omt * 1.0f + t * 0.5f, omt * 1.0f + t * 0.7f, omt * 1.0f + t * 1.0f};
}

// ---------------------------------------------------------------- scene view
struct Scene {
    const float* tris; int nt;
    const float* nodes; int nn;
    const float* mats; int nm;
    const float* spheres; int ns;
};
struct Counters { uint64_t seg = 0, nodes = 0, tri_tests = 0, sphere_tests = 0, hits = 0; };

float hit_sphere(V3 o, V3 d, const float* sp) {                // :209-226
    V3 c = ld3(sp);
    float r = sp[3];
    V3 oc = sub(o, c);
    float a = dot(d, d);
    float half_b = dot(oc, d);
    float cc = dot(oc, oc) - r * r;
    float disc = half_b * half_b - a * cc;
    if (disc < 0.0f) return -1.0f;
    return (-half_b - std::sqrt(disc)) / a;
}

float hit_triangle(V3 o, V3 d, const float* tri, V3& normal) { // :274-307 (live test)
    V3 v0 = ld3(tri), v1 = ld3(tri + 4), v2 = ld3(tri + 8);
    V3 a = sub(v1, v0), b = sub(v2, v0);
    V3 n = normalize(cross(a, b));
    normal = n;
    float dd = -dot(n, v0);
    float t = -(dot(n, o) + dd) / dot(n, d);
    if (t < 0.0f) return -1.0f;
    V3 p = add(o, muls(d, t));
    V3 e0 = sub(v1, v0), e1 = sub(v2, v1), e2 = sub(v0, v2);
    V3 c0 = sub(p, v0), c1 = sub(p, v1), c2 = sub(p, v2);
    if (dot(n, cross(e0, c0)) > 0.0f && dot(n, cross(e1, c1)) > 0.0f &&
        dot(n, cross(e2, c2)) > 0.0f)
        return t;
    return -1.0f;
}

// RayIntersectsTriangle :228-272 -- Moller-Trumbore, EPSILON 1e-7.  Dead code in the
// reference (hit_triangle is the live test); the opt-in PT_FLAG_MOLLER_TRUMBORE (flags bit 5)
// mode of the build runs it in hit_triangle's place.
float mt_triangle(V3 o, V3 d, const float* tri, V3& normal) {
    const float EPS = 0.0000001f;
    V3 v0 = ld3(tri), v1 = ld3(tri + 4), v2 = ld3(tri + 8);
    V3 e1 = sub(v1, v0), e2 = sub(v2, v0);
    V3 h = cross(d, e2);
    float a = dot(e1, h);
    if (a > -EPS && a < EPS) return -1.0f;
    float f = 1.0f / a;
    V3 s = sub(o, v0);
    float u = f * dot(s, h);
    if (u < 0.0f || u > 1.0f) return -1.0f;
    V3 q = cross(s, e1);
    float v = f * dot(d, q);
    if (v < 0.0f || u + v > 1.0f) return -1.0f;
    float t = f * dot(e2, q);
    if (t > EPS) {
        normal = normalize(cross(e1, e2));
        return t;
    }
    return -1.0f;
}

bool bvh_intersect(const float* b, V3 o, V3 d, float cur_t) {  // :309-365
    float tmin = (b[0] - o.x) / d.x;
    float tmax = (b[4] - o.x) / d.x;
    if (tmin > tmax) std::swap(tmin, tmax);
    float tymin = (b[1] - o.y) / d.y;
    float tymax = (b[5] - o.y) / d.y;
    if (tymin > tymax) std::swap(tymin, tymax);
    if ((tmin > tymax) || (tymin > tmax)) return false;
    if (tymin > tmin) tmin = tymin;
    if (tymax < tmax) tmax = tymax;
    float tzmin = (b[2] - o.z) / d.z;
    float tzmax = (b[6] - o.z) / d.z;
    if (tzmin > tzmax) std::swap(tzmin, tzmax);
    if ((tmin > tzmax) || (tzmin > tmax)) return false;
    if (tzmin > tmin) tmin = tzmin;
    if (tzmax < tmax) tmax = tzmax;
    (void)tmax;
    if (tmin > cur_t) return false;
    return true;
}

// :367-432
void ray_collision(const Scene& sc, V3 o, V3 d, V3& normal, V3& hit_point, bool& hit,
                   int& mat_index, int flags, Counters* cnt) {
    float t = std::numeric_limits<float>::infinity();
    for (int si = 0; si < ((flags & 4) ? 0 : sc.ns); si++) {
        const float* sp = sc.spheres + 8 * si;
        float ht = hit_sphere(o, d, sp);
        if (cnt) cnt->sphere_tests++;
        if (ht > 0.0001f && ht < t) {
            V3 pn = normalize(sub(add(o, muls(d, ht)), ld3(sp)));
            if (dot(pn, d) > 0.0f) pn = muls(pn, -1.0f);
            hit = true;
            t = ht;
            normal = pn;
            hit_point = add(o, muls(d, ht));
            mat_index = (int)sp[4];
        }
    }
    if (sc.nn <= 0 || (flags & 8)) return;
    V3 rn, rn2;
    for (int bi = 0; bi > -1;) {
        const float* b = sc.nodes + 12 * bi;
        bool hb = bvh_intersect(b, o, d, t);
        if (cnt) cnt->nodes++;
        int next = hb ? (int)b[10] : (int)b[11];
        if (hb && (b[8] > -1.0f)) {
            if (cnt) cnt->tri_tests += 2;
            int t0 = (int)b[8], t1 = (int)b[9];
            float h1, h2;
            if (flags & 32) {
                h1 = mt_triangle(o, d, sc.tris + 16 * t0, rn);
                h2 = mt_triangle(o, d, sc.tris + 16 * t1, rn2);
            } else {
                h1 = hit_triangle(o, d, sc.tris + 16 * t0, rn);
                h2 = hit_triangle(o, d, sc.tris + 16 * t1, rn2);
            }
            if (h1 > 0.0001f && h1 < t && (h1 < h2 || h2 < 0.0001f)) {
                if (dot(rn, d) > 0.0f) rn = muls(rn, -1.0f);
                hit = true;
                t = h1;
                normal = rn;
                hit_point = add(o, muls(d, h1));
                mat_index = (int)sc.tris[16 * t0 + 12];
            } else if (h2 > 0.0001f && h2 < t) {
                if (dot(rn2, d) > 0.0f) rn2 = muls(rn2, -1.0f);
                hit = true;
                t = h2;
                normal = rn2;
                hit_point = add(o, muls(d, h2));
                mat_index = (int)sc.tris[16 * t1 + 12];
            }
        }
        bi = next;
    }
}

// :434-501
// flags: bit0 antiAlias off, bit1 EnvironmentEnabled off, bit2 render_spheres off,
// bit3 render_triangles off (computeShader.c:77-82 compile-time toggles; 0 = reference),
// bit5 Moller-Trumbore triangle test (the reference's dead RayIntersectsTriangle).
V3 trace(const Scene& sc, V3 o, V3 d, uint32_t& state, int max_bounce, int mode, int flags,
         Counters* cnt) {
    V3 incoming = v3(0, 0, 0);
    V3 ray_color = v3(1, 1, 1);
    V3 normal = v3(0, 0, 0), hit_point = v3(0, 0, 0);
    int mat = 0;
    for (int i = 0; i <= max_bounce; i++) {
        bool hit = false;
        ray_collision(sc, o, d, normal, hit_point, hit, mat, flags, cnt);
        if (cnt) { cnt->seg++; if (hit) cnt->hits++; }
        if (hit && length(ray_color) > 0.01f) {
            if (mode == 2) return muls(add(normal, v3(1, 1, 1)), 0.5f);
            if (mode == 4) {
                float s = length(sub(hit_point, o));
                float dist = 1.0f - std::sqrt(s + 1.0f) / (s + 1.0f);
                float q = dist * dist;
                return v3(q, q, q);
            }
            o = hit_point;
            V3 diffuse_dir = normalize(add(normal, random_unit_vector(state)));
            // reflect(I, N) = I - 2*dot(N, I)*N
            float k = 2.0f * dot(normal, d);
            V3 specular_dir = normalize(sub(d, muls(normal, k)));
            const float* m = sc.mats + 16 * mat;
            float spec_prob = m[14], smooth = m[13], emis_strength = m[12];
            if (mode == 3) return ld3(m);
            float is_spec = 0.0f;
            if (spec_prob > random01(state)) is_spec = 1.0f;
            d = mixv(diffuse_dir, specular_dir, smooth * is_spec);
            V3 emitted = muls(ld3(m + 4), emis_strength);
            incoming = add(incoming, mul(emitted, ray_color));
            ray_color = mul(ray_color, mixv(ld3(m), ld3(m + 8), is_spec));
        } else {
            V3 env = (flags & 2) ? v3(0, 0, 0) : environment_light(d);
            incoming = add(incoming, mul(env, ray_color));
            break;
        }
    }
    return incoming;
}

struct Camera { V3 pos, fwd, right, up; };

// :517-522 camera basis (per dispatch constant)
Camera make_camera(const float* cam, int W, int H) {
    Camera c;
    c.pos = ld3(cam);
    c.fwd = normalize(ld3(cam + 4));
    c.right = normalize(cross(c.fwd, v3(0, 0, 1)));
    c.up = divs(muls(normalize(cross(c.right, c.fwd)), (float)H), (float)W);
    return c;
}

// One sample (one dispatch invocation) for pixel (x, y) at `frame` -> rgb  (:505-546)
// rpp = raysPerPixel (computeShader.c:507, 1 in the reference): pixel = 0 + sum, / rpp.
V3 sample_pixel(const Scene& sc, const Camera& c, int x, int y, int W, int H, int frame,
                int max_bounce, int mode, int flags, int rpp, Counters* cnt) {
    uint32_t pix = (uint32_t)y * 831266u + (uint32_t)x * 923766u;
    uint32_t state = pix + (uint32_t)frame * 719393u;
    V3 pixel = v3(0, 0, 0);
    for (int r = 0; r < rpp; r++) {
        float ax = 0.0f, ay = 0.0f;
        if (!(flags & 1)) {
            ax = random01(state);
            ay = random01(state);
        }
        float u = ((float)x + ax) / (float)W - 0.5f;
        float v = ((float)y + ay) / (float)H - 0.5f;
        V3 d = normalize(add(add(c.fwd, muls(c.right, u)), muls(c.up, v)));
        pixel = add(pixel, trace(sc, c.pos, d, state, max_bounce, mode, flags, cnt));
    }
    return divs(pixel, (float)rpp);
}

// :548-553  acc = prev*((f-1)/f) + (rgb,1)/f, or plain store.
inline void accumulate(float* px, V3 rgb, int frame, bool acc) {
    if (acc) {
        float ff = (float)frame;
        float w = (ff - 1.0f) / ff;
        px[0] = px[0] * w + rgb.x / ff;
        px[1] = px[1] * w + rgb.y / ff;
        px[2] = px[2] * w + rgb.z / ff;
        px[3] = px[3] * w + 1.0f / ff;
    } else {
        px[0] = rgb.x; px[1] = rgb.y; px[2] = rgb.z; px[3] = 1.0f;
    }
}

// ================================================================ loader (geometry_loader.h)
// Restates load_vertex_data(): MTL first (8 lines per newmtl block), then OBJ.
// istream semantics: a failed extraction stores 0 and later extractions are skipped;
// never-written fields are 0 (build decision).
struct LoadResult { std::vector<float> tris, mats; int err = 0; std::string msg; };

bool read_line128(std::istream& in, std::string& line, bool& too_long) {
    too_long = false;
    if (!std::getline(in, line)) return false;
    // getline(buf, 128) stores at most 127 chars; a longer line sets failbit and the
    // reference's `while (!eof())` loop never terminates -> reported as an error here.
    if (line.size() > 127) too_long = true;
    return true;
}

LoadResult load_vertex_data(const char* obj_path, const char* mtl_path) {
    LoadResult R;
    std::unordered_map<std::string, int> mmap;
    std::ifstream m(mtl_path);
    if (!m.is_open()) { R.err = -2; R.msg = "Failed to open material file"; return R; }
    std::string line;
    bool tl;
    while (read_line128(m, line, tl)) {
        if (tl) { R.err = -3; R.msg = "line longer than 127 chars"; return R; }
        std::istringstream s(line);
        std::string ident, name;
        s >> ident >> name;
        if (ident == "newmtl") {
            float col[4] = {0, 0, 0, 0}, emi[4] = {0, 0, 0, 0}, spc[4] = {0, 0, 0, 0},
                  dat[4] = {0, 0, 0, 0};
            for (int k = 0; k < 8; k++) {
                std::string ld;
                if (!read_line128(m, ld, tl)) ld.clear();
                if (tl) { R.err = -3; R.msg = "line longer than 127 chars"; return R; }
                std::istringstream sd(ld);
                std::string thr;
                if (ld.size() >= 2 && ld[0] == 'N' && ld[1] == 's') {
                    float z = 0; sd >> thr >> z;   // a failed parse stores 0
                    dat[2] = (float)((double)z / 1000.0);
                } else if (ld.size() >= 2 && ld[0] == 'K') {
                    float* dst = nullptr;
                    if (ld[1] == 'e') dst = emi;
                    if (ld[1] == 'd') dst = col;
                    if (ld[1] == 's') dst = spc;
                    if (dst) {
                        float a = 0, b = 0, c = 0;
                        sd >> thr;
                        if (sd >> a) { if (sd >> b) { sd >> c; } }
                        dst[0] = a; dst[1] = b; dst[2] = c;
                    }
                }
            }
            if (dat[2] > 0) dat[1] = 1.0f;
            dat[0] = 7.5f;
            for (float* p : {col, emi, spc, dat}) R.mats.insert(R.mats.end(), p, p + 4);
            mmap[name] = (int)(R.mats.size() / 16) - 1;
        }
    }
    std::ifstream f(obj_path);
    if (!f.is_open()) { R.err = -2; R.msg = "Failed to open vertex file"; return R; }
    std::vector<float> verts;
    std::string cur;
    while (read_line128(f, line, tl)) {
        if (tl) { R.err = -3; R.msg = "line longer than 127 chars"; return R; }
        if (line.empty()) continue;
        std::istringstream s(line);
        if (line[0] == 'u') { std::string pre; s >> pre >> cur; }
        if (line[0] == 'v') {
            char id; float x = 0, y = 0, z = 0;
            s >> id;
            if (s >> x) { if (s >> y) { s >> z; } }
            verts.push_back(x); verts.push_back(y); verts.push_back(z);
        }
        if (line[0] == 'f') {
            char id; long long fi[3] = {0, 0, 0};
            s >> id;
            bool ok = false;
            if (s >> fi[0]) { if (s >> fi[1]) { if (s >> fi[2]) ok = true; } }
            long long nv = (long long)verts.size() / 3;
            if (!ok || fi[0] < 1 || fi[1] < 1 || fi[2] < 1 || fi[0] > nv || fi[1] > nv ||
                fi[2] > nv) {
                R.err = -4; R.msg = "face index out of range"; return R;
            }
            int midx = mmap[cur];  // unknown name -> inserted as 0 (reference behaviour)
            for (int k = 0; k < 3; k++) {
                const float* v = &verts[3 * (fi[k] - 1)];
                R.tris.push_back(v[0]); R.tris.push_back(v[1]); R.tris.push_back(v[2]);
                R.tris.push_back(0.0f);
            }
            R.tris.push_back((float)midx); R.tris.push_back(0); R.tris.push_back(0);
            R.tris.push_back(0);
        }
    }
    return R;
}

// ================================================================ BVH (bvh.h:21-268)
// Literal restatement with value-copied vectors, std::stable_sort (the reference's
// std::sort is unstable: ties would be implementation-defined) and
// the O(N) std::find per leaf.  Quadratic: use only on test-sized inputs.
struct Tri { float v[16]; };
bool tri_eq(const Tri& a, const Tri& b) {
    for (int i = 0; i < 16; i++) if (!(a.v[i] == b.v[i])) return false;
    return true;
}
struct Node { float mn[4], mx[4], data[4]; };

void expand(Node& b, const Tri& t) {
    for (int a = 0; a < 3; a++) {
        for (int vi = 0; vi < 3; vi++) {
            float c = t.v[4 * vi + a];
            if (c < b.mn[a]) b.mn[a] = c;
            if (c > b.mx[a]) b.mx[a] = c;
        }
    }
}
Node empty_node() {
    Node n;
    for (int i = 0; i < 4; i++) {
        n.mn[i] = std::numeric_limits<float>::infinity();
        n.mx[i] = -std::numeric_limits<float>::infinity();
        n.data[i] = 0.0f;
    }
    return n;
}
double surface_area(const Node& b) {
    double x = (float)(b.mx[0] - b.mn[0]);
    double y = (float)(b.mx[1] - b.mn[1]);
    double z = (float)(b.mx[2] - b.mn[2]);
    return 2.0 * (x * y + y * z + x * z);
}
bool compare_tris(const Tri& a, const Tri& b, int axis) {
    double c1 = (double)(float)((a.v[axis] + a.v[4 + axis]) + a.v[8 + axis]) / 3.0;
    double c2 = (double)(float)((b.v[axis] + b.v[4 + axis]) + b.v[8 + axis]) / 3.0;
    return c1 < c2;
}

// find_split (bvh.h:173-218).  Returns false when no candidate has a finite cost below
// +inf (degenerate: SA == 0), where the reference would recurse on an empty vector;
// the build then splits at n/2 of the z-sorted order (documented deviation).
bool find_split(std::vector<Tri> tris, std::vector<Tri>& s1, std::vector<Tri>& s2) {
    Node overall = empty_node();
    for (auto& t : tris) expand(overall, t);
    double SA = surface_area(overall);
    double min_cost = std::numeric_limits<double>::infinity();
    bool found = false;
    const double Ci = 1.0, Ct = 1.0;
    for (int axis = 0; axis < 3; axis++) {
        std::stable_sort(tris.begin(), tris.end(),
                         [axis](const Tri& a, const Tri& b) { return compare_tris(a, b, axis); });
        size_t n = tris.size();
        for (int split = 1; (size_t)split < n; split += (int)(n / 60 + 1)) {
            Node b1 = empty_node(), b2 = empty_node();
            for (int i = 0; i < split; i++) expand(b1, tris[i]);
            for (size_t i = split; i < n; i++) expand(b2, tris[i]);
            double SA1 = surface_area(b1), SA2 = surface_area(b2);
            double cost = Ct + (SA1 / SA) * split * Ci + (SA2 / SA) * (double)(n - split) * Ci;
            if (cost < min_cost) {
                s1.assign(tris.begin(), tris.begin() + split);
                s2.assign(tris.begin() + split, tris.end());
                min_cost = cost;
                found = true;
            }
        }
    }
    if (!found) {
        size_t h = tris.size() / 2;
        s1.assign(tris.begin(), tris.begin() + h);
        s2.assign(tris.begin() + h, tris.end());
    }
    return found;
}

void build_helper(const std::vector<Tri>& ref, std::vector<Tri> tris, std::vector<Node>& bounds,
                  int insert) {
    Node overall = empty_node();
    for (auto& t : tris) expand(overall, t);
    if (tris.size() <= 2) {
        auto i0 = std::find_if(ref.begin(), ref.end(), [&](const Tri& r) { return tri_eq(r, tris[0]); });
        auto i1 = std::find_if(ref.begin(), ref.end(),
                               [&](const Tri& r) { return tri_eq(r, tris[tris.size() - 1]); });
        overall.data[0] = (float)(i0 - ref.begin());
        overall.data[1] = (float)(i1 - ref.begin());
        overall.data[3] = -1.0f;
        overall.data[2] = -1.0f;
        bounds[insert] = overall;
        return;
    }
    std::vector<Tri> left, right;
    find_split(tris, left, right);
    bounds.push_back(empty_node());
    bounds.push_back(empty_node());
    overall.data[0] = -1.0f;   // build decision: internal nodes carry tri0 = tri1 = -1
    overall.data[1] = -1.0f;
    overall.data[2] = (float)(bounds.size() - 2);
    overall.data[3] = (float)(bounds.size() - 1);
    int l = (int)overall.data[2], r = (int)overall.data[3];
    build_helper(ref, left, bounds, l);
    build_helper(ref, right, bounds, r);
    bounds[insert] = overall;
}

void build_links(const std::vector<Node>& tree, std::vector<Node>& mod, int cur, int next_right) {
    if (tree[cur].data[3] > -1.0f) {
        int c1 = (int)tree[cur].data[2], c2 = (int)tree[cur].data[3];
        mod[cur].data[2] = (float)c1;
        mod[cur].data[3] = (float)next_right;
        build_links(tree, mod, c1, c2);
        build_links(tree, mod, c2, next_right);
    } else {
        mod[cur].data[2] = (float)next_right;
        mod[cur].data[3] = (float)next_right;
    }
}

}  // namespace

// ===================================================================== C ABI (ctypes)
extern "C" {

float oracle_logf(float x) { return o_logf(x); }
float oracle_mt_triangle(const float* o, const float* d, const float* tri, float* normal) {
    V3 n = v3(0, 0, 0);
    float t = mt_triangle(v3(o[0], o[1], o[2]), v3(d[0], d[1], d[2]), tri, n);
    normal[0] = n.x; normal[1] = n.y; normal[2] = n.z;
    return t;
}
float oracle_hit_triangle(const float* o, const float* d, const float* tri, float* normal) {
    V3 n = v3(0, 0, 0);
    float t = hit_triangle(v3(o[0], o[1], o[2]), v3(d[0], d[1], d[2]), tri, n);
    normal[0] = n.x; normal[1] = n.y; normal[2] = n.z;
    return t;
}
float oracle_cosf(float x) { return o_cosf(x); }

// Batch forms for exhaustive checks.
void oracle_logf_n(const float* x, float* y, long long n) {
    for (long long i = 0; i < n; i++) y[i] = o_logf(x[i]);
}
void oracle_cosf_n(const float* x, float* y, long long n) {
    for (long long i = 0; i < n; i++) y[i] = o_cosf(x[i]);
}

// Draw `n` successive random() values from `state`.
void oracle_random_seq(unsigned state, int n, float* out, unsigned* raw) {
    uint32_t s = state;
    for (int i = 0; i < n; i++) {
        uint32_t s2 = s;
        uint32_t r = next_random(s2);
        if (raw) raw[i] = r;
        out[i] = random01(s);
    }
}
unsigned oracle_seed(int x, int y, int frame) {
    uint32_t pix = (uint32_t)y * 831266u + (uint32_t)x * 923766u;
    return pix + (uint32_t)frame * 719393u;
}

// Returns 0 and fills counts; on error returns <0.  Pass null buffers to query sizes.
int oracle_load_obj(const char* obj, const char* mtl, float* tris, int max_tris, int* n_tris,
                    float* mats, int max_mats, int* n_mats) {
    LoadResult R = load_vertex_data(obj, mtl);
    if (R.err) return R.err;
    int nt = (int)(R.tris.size() / 16), nm = (int)(R.mats.size() / 16);
    *n_tris = nt;
    *n_mats = nm;
    if (tris) {
        if (nt > max_tris) return -1;
        std::memcpy(tris, R.tris.data(), R.tris.size() * 4);
    }
    if (mats) {
        if (nm > max_mats) return -1;
        std::memcpy(mats, R.mats.data(), R.mats.size() * 4);
    }
    return 0;
}

// buildSAHTree (bvh.h:255-268).  nodes: capacity 2*n_tris nodes of 12 floats.
int oracle_build_bvh(const float* tris_in, int n_tris, float* nodes_out, int max_nodes,
                     int* n_nodes) {
    if (n_tris <= 0) { *n_nodes = 0; return -1; }   // the reference indexes triangles[0]
    std::vector<Tri> tris(n_tris);
    for (int i = 0; i < n_tris; i++) std::memcpy(tris[i].v, tris_in + 16 * i, 64);
    std::vector<Node> h;
    h.push_back(empty_node());
    build_helper(tris, tris, h, 0);
    std::vector<Node> mod = h;
    build_links(h, mod, 0, -1);
    *n_nodes = (int)mod.size();
    if ((int)mod.size() > max_nodes) return -1;
    for (size_t i = 0; i < mod.size(); i++) std::memcpy(nodes_out + 12 * i, &mod[i], 48);
    return 0;
}

// setupBuffers() built-ins (ogl_path_trace.h:415-453, 498-501): writes 5 materials
// (80 floats) and the one metal sphere (8 floats) for `n_loaded` loaded materials.
void oracle_builtins(int n_loaded, float* mats5, float* sphere) {
    const float M[5][16] = {
        {0, 0, 0, 1, 0.99f, 0.95f, 0.78f, 1, 0, 0, 0, 0, 1.5f, 0, 0, 0},          // light
        {1, 0.39f, 0.28f, 1, 0, 0, 0, 1, 1, 1, 1, 1, 0, 1, 0.18f, 0},           // spec
        {1, 0.5f, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 0, 1, 0.1f, 0},                 // diffuse
        {1, 0.9f, 0.9f, 1, 0, 0, 0, 1, 0, 0, 0, 1, 0, 0, 0, 0},                 // ground
        {0.9f, 0.9f, 0.1f, 1, 0, 0, 0, 1, 1, 1, 1, 1, 0, 0.9f, 0.91f, 0},       // metal
    };
    std::memcpy(mats5, M, sizeof(M));
    const float S[8] = {-0.5f, 3.0f, 1.0f, 0.8f, (float)n_loaded + 4.0f, 0, 0, 0};
    std::memcpy(sphere, S, sizeof(S));
}

// Full-frame render: n_frames dispatches, frames frame_first.., the first with
// accumulate = acc_first, the rest accumulate = 1.  accum: W*H*4 floats, row 0 = bottom.
// counters (optional): [segments, node visits, tri tests, sphere tests, hits].
int oracle_render(const float* tris, int nt, const float* nodes, int nn, const float* mats,
                  int nm, const float* spheres, int ns, const float* cam, int W, int H,
                  int max_bounce, int mode, int flags, int rpp, int frame_first, int n_frames,
                  int acc_first, float* accum, int threads, unsigned long long* counters) {
    Scene sc{tris, nt, nodes, nn, mats, nm, spheres, ns};
    Camera c = make_camera(cam, W, H);
    if (threads < 1) threads = 1;
    std::atomic<int> next_row{0};
    std::vector<Counters> cs(threads);
    auto work = [&](int tid) {
        Counters* cnt = counters ? &cs[tid] : nullptr;
        for (;;) {
            int y = next_row.fetch_add(1);
            if (y >= H) break;
            for (int x = 0; x < W; x++) {
                float* px = accum + 4 * ((size_t)y * W + x);
                for (int k = 0; k < n_frames; k++) {
                    int f = frame_first + k;
                    V3 rgb = sample_pixel(sc, c, x, y, W, H, f, max_bounce, mode, flags, rpp, cnt);
                    accumulate(px, rgb, f, k == 0 ? acc_first == 1 : true);
                }
            }
        }
    };
    std::vector<std::thread> th;
    for (int t = 1; t < threads; t++) th.emplace_back(work, t);
    work(0);
    for (auto& t : th) t.join();
    if (counters) {
        for (int i = 0; i < 5; i++) counters[i] = 0;
        for (auto& q : cs) {
            counters[0] += q.seg; counters[1] += q.nodes; counters[2] += q.tri_tests;
            counters[3] += q.sphere_tests; counters[4] += q.hits;
        }
    }
    return 0;
}

// Same semantics for a pixel subset: px_rgba holds the n pixels' prior values (in/out).
int oracle_render_pixels(const float* tris, int nt, const float* nodes, int nn,
                         const float* mats, int nm, const float* spheres, int ns,
                         const float* cam, int W, int H, int max_bounce, int mode, int flags,
                         int rpp, int frame_first, int n_frames, int acc_first, const int* xs,
                         const int* ys, int n, float* px_rgba, int threads,
                         unsigned long long* counters) {
    Scene sc{tris, nt, nodes, nn, mats, nm, spheres, ns};
    Camera c = make_camera(cam, W, H);
    if (threads < 1) threads = 1;
    std::atomic<int> next{0};
    std::vector<Counters> cs(threads);
    auto work = [&](int tid) {
        Counters* cnt = counters ? &cs[tid] : nullptr;
        for (;;) {
            int i = next.fetch_add(1);
            if (i >= n) break;
            float* px = px_rgba + 4 * (size_t)i;
            for (int k = 0; k < n_frames; k++) {
                int f = frame_first + k;
                V3 rgb = sample_pixel(sc, c, xs[i], ys[i], W, H, f, max_bounce, mode, flags, rpp, cnt);
                accumulate(px, rgb, f, k == 0 ? acc_first == 1 : true);
            }
        }
    };
    std::vector<std::thread> th;
    for (int t = 1; t < threads; t++) th.emplace_back(work, t);
    work(0);
    for (auto& t : th) t.join();
    if (counters) {
        for (int i = 0; i < 5; i++) counters[i] = 0;
        for (auto& q : cs) {
            counters[0] += q.seg; counters[1] += q.nodes; counters[2] += q.tri_tests;
            counters[3] += q.sphere_tests; counters[4] += q.hits;
        }
    }
    return 0;
}

// ACES film curve (screenQuadFrag.c:12-26) -> RGBA8, alpha 255.  Rounding to 8 bits is
// the build's choice (the reference hands the float to the GL framebuffer): round-half-up
// of v*255.
void oracle_aces_rgba8(const float* rgba, int n_pixels, unsigned char* out) {
    for (int i = 0; i < n_pixels; i++) {
        for (int c = 0; c < 3; c++) {
            float v = rgba[4 * i + c];
            float tm = (v * (2.51f * v + 0.03f)) / (v * (2.43f * v + 0.59f) + 0.14f);
            tm = tm < 0.0f ? 0.0f : (tm > 1.0f ? 1.0f : tm);   // clamp; NaN -> passes through
            if (!(tm == tm)) tm = 0.0f;
            out[4 * i + c] = (unsigned char)(int)(tm * 255.0f + 0.5f);
        }
        out[4 * i + 3] = 255;
    }
}

// The interactive loop of run() (ogl_path_trace.h:160-204) with its two GLFW callbacks
// (handleMovementInput :258-299, cursorPosCallback :332-364) and updateCameraBuffer
// (:301-328), replayed from an event list:
//   kind[i] 0: one loop iteration at glfwGetTime() = a[i]; 1: key callback (key[i],
//   action[i]); 2: cursor callback (a[i], b[i]).
// The loop ends early once Escape was pressed (glfwWindowShouldClose, :160).  Per frame
// the dispatch parameters are written: cam_out 12 floats {position, direction, 0},
// fia_out 3 ints {frame, accumulate, displayMode}.  Returns the number of frames.
// glm is restated from its generic (non-SIMD) code: vec4 dot = (xx + yy) + (zz + ww),
// normalize = v * (1 / sqrt(dot)), radians(d) = d * 0.01745329251994329576923690768489.
struct GVec4 { float x, y, z, w; };

int oracle_viewer_replay(int n_events, const int* kind, const double* a, const double* b, const int* key,
                         const int* action, const float* cam0, int display_mode0, float moveSpeed,
                         float rotSpeed, int userDefinedAccumulate, int max_frames, float* cam_out,
                         int* fia_out) {
    const float PI = 3.141592f;
    GVec4 camera_position = {0.0f, -6.0f, 1.0f, 0.0f}, camera_direction = {0.0f, 1.0f, 0.0f, 0.0f};
    if (cam0) {
        camera_position = {cam0[0], cam0[1], cam0[2], cam0[3]};
        camera_direction = {cam0[4], cam0[5], cam0[6], cam0[7]};
    }
    bool mF = false, mB = false, mL = false, mR = false, mU = false, mD = false, mC = false;
    bool window_should_close = false;
    double pxpos = 0, pypos = 0;
    int displayMode = display_mode0, accumulate = 0, frameCount = 0;
    float deltaTime = 0.0f, lastFrameTime = 0.0f;
    int frames = 0;
    bool first = true;
    for (int i = 0; i < n_events; i++) {
        if (kind[i] == 1) {                      // handleMovementInput
            const int k = key[i], act = action[i];
            const int prevDisplayMode = displayMode;
            if (k == 49) displayMode = 1;
            if (k == 50) displayMode = 2;
            if (k == 51) displayMode = 3;
            if (k == 52) displayMode = 4;
            if (prevDisplayMode != displayMode) mC = true;
            if (k == 87) { if (act == 1) mF = true; if (act == 0) mF = false; }
            if (k == 65) { if (act == 1) mL = true; if (act == 0) mL = false; }
            if (k == 83) { if (act == 1) mB = true; if (act == 0) mB = false; }
            if (k == 68) { if (act == 1) mR = true; if (act == 0) mR = false; }
            if (k == 32) { if (act == 1) mU = true; if (act == 0) mU = false; }
            if (k == 340) { if (act == 1) mD = true; if (act == 0) mD = false; }
            if (k == 256) window_should_close = true;
            continue;
        }
        if (kind[i] == 2) {                      // cursorPosCallback
            const double xpos = a[i], ypos = b[i];
            mC = true;
            double rotationAroundZ = ((pxpos - xpos) * 0.01745329251994329576923690768489) * (double)rotSpeed;
            double rotationAroundHoriz = ((pypos - ypos) * 0.01745329251994329576923690768489) * (double)rotSpeed;
            float lz2 = camera_direction.x * camera_direction.x + camera_direction.y * camera_direction.y;
            double lengthFromZPerspective = (double)sqrtf(lz2);
            double currentZAngle = (double)atan2f(camera_direction.y, camera_direction.x);
            double newZAngle = currentZAngle + rotationAroundZ;
            float l2 = camera_direction.x * camera_direction.x + camera_direction.y * camera_direction.y;
            l2 = l2 + camera_direction.z * camera_direction.z;
            double length = (double)sqrtf(l2);
            double currentHAngle = atan2((double)camera_direction.z, lengthFromZPerspective);
            double newHAngle = currentHAngle + rotationAroundHoriz;
            const double half_pi = (double)PI / 2.0, neg_half_pi = (double)(-PI) / 2.0;
            if (newHAngle > half_pi || newHAngle < neg_half_pi) newHAngle = currentHAngle;
            double newZ = length * sin(newHAngle);
            double newXYLength = length * cos(newHAngle);
            double newX = newXYLength * cos(newZAngle);
            double newY = newXYLength * sin(newZAngle);
            camera_direction = {(float)newX, (float)newY, (float)newZ, 0.0f};
            pxpos = xpos;
            pypos = ypos;
            continue;
        }
        // one loop iteration
        if (window_should_close || frames >= max_frames) break;
        if (!first) {                            // tail of the previous iteration
            accumulate = userDefinedAccumulate;
            if (mF || mR || mB || mL || mU || mD || mC) {
                accumulate = 0;
                frameCount = 0;
            }
            mC = false;
        }
        first = false;
        // updateCameraBuffer
        GVec4 t = {camera_direction.x - 0.0f, camera_direction.y - 0.0f, camera_direction.z - camera_direction.z,
                   camera_direction.w - 0.0f};
        float dd = (t.x * t.x + t.y * t.y) + (t.z * t.z + t.w * t.w);
        float inv = 1.0f / sqrtf(dd);
        GVec4 forward = {t.x * inv, t.y * inv, t.z * inv, t.w * inv};
        // cross(forward3, (0,0,1))
        GVec4 right = {forward.y * 1.0f - 0.0f * forward.z, forward.z * 0.0f - 1.0f * forward.x,
                       forward.x * 0.0f - 0.0f * forward.y, 0.0f};
        GVec4 up = {0.0f, 0.0f, 1.0f, 0.0f};
        auto step = [&](const GVec4& v, float sign) {
            const float sx = (v.x * moveSpeed) * deltaTime, sy = (v.y * moveSpeed) * deltaTime;
            const float sz = (v.z * moveSpeed) * deltaTime, sw = (v.w * moveSpeed) * deltaTime;
            if (sign > 0) {
                camera_position = {camera_position.x + sx, camera_position.y + sy, camera_position.z + sz,
                                   camera_position.w + sw};
            } else {
                camera_position = {camera_position.x - sx, camera_position.y - sy, camera_position.z - sz,
                                   camera_position.w - sw};
            }
        };
        if (mF) step(forward, 1.0f);
        if (mL) step(right, -1.0f);
        if (mB) step(forward, -1.0f);
        if (mR) step(right, 1.0f);
        if (mU) step(up, 1.0f);
        if (mD) step(up, -1.0f);
        frameCount++;
        float currentTime = (float)a[i];
        deltaTime = currentTime - lastFrameTime;
        lastFrameTime = currentTime;
        float* c = cam_out + 12 * frames;
        const float buf[12] = {camera_position.x, camera_position.y, camera_position.z, camera_position.w,
                               camera_direction.x, camera_direction.y, camera_direction.z, camera_direction.w,
                               0.0f, 0.0f, 0.0f, 0.0f};
        std::memcpy(c, buf, sizeof(buf));
        fia_out[3 * frames + 0] = frameCount;
        fia_out[3 * frames + 1] = accumulate;
        fia_out[3 * frames + 2] = displayMode;
        frames++;
    }
    return frames;
}

}  // extern "C"
