// pt_scene.cpp -- host scene ingest: OBJ/MTL loader, SAH BVH builder, built-in assembly.
//
// Product code (C++17, no GPU).  Re-designed from the reference's host pipeline:
//   geometry_loader.h:15-142   load_vertex_data  -> pt_scene_load_obj   (single-pass buffer parser)
//   bvh.h:173-268              buildSAHTree      -> pt_bvh_build        (index-based, O(n log^2 n))
//   ogl_path_trace.h:415-507   setupBuffers      -> pt_scene_add_builtins
//
// The builder reproduces the reference topology exactly (same node numbering, same
// split choices, same leaf triangle indices) but replaces the reference's per-candidate
// box re-expansion (O(60 n) per axis) with prefix/suffix boxes and its O(N) std::find per
// leaf (O(N^2) overall) with a first-occurrence hash map.  Sorting is std::stable_sort
// chained x -> y -> z exactly like the reference's three successive std::sort calls on
// one vector (the reference's unstable sort leaves ties implementation-defined; the
// build pins them stable).  Build with -ffp-contract=off.
#include "../../include/pt_scene.h"
#include "../../include/pt_api.h"

#include <algorithm>
#include <cerrno>
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <limits>
#include <string>
#include <unordered_map>
#include <vector>

struct pt_scene {
    std::vector<float> tris;     // 16 floats / tri
    std::vector<float> mats;     // 16 floats / material
    std::vector<float> spheres;  // 8 floats / sphere
    std::vector<float> nodes;    // 12 floats / node
    int n_loaded_mats = 0;
    bool builtins = false;
    std::string err;
};

namespace {

// ---------------------------------------------------------------- text scanning
// Mirrors the istream extraction semantics the reference relies on: whitespace-delimited
// tokens; a failed numeric extraction yields 0 and poisons the rest of the line.
struct Cursor {
    const char* p;
    const char* e;
    bool fail = false;
    static bool ws(char c) { return c == ' ' || c == '\t' || c == '\r' || c == '\v' || c == '\f' || c == '\n'; }
    void skip() { while (p < e && ws(*p)) ++p; }
    bool token(std::string& out) {          // operator>>(std::string)
        if (fail) return false;
        skip();
        if (p >= e) { fail = true; return false; }
        const char* s = p;
        while (p < e && !ws(*p)) ++p;
        out.assign(s, p - s);
        return true;
    }
    bool ch(char& c) {                      // operator>>(char)
        if (fail) return false;
        skip();
        if (p >= e) { fail = true; return false; }
        c = *p++;
        return true;
    }
    // operator>>(float): accumulate [+-]digits[.digits][(e|E)[+-]digits] then strtof on it.
    bool num_f(float& v) {
        if (fail) return false;
        skip();
        const char* s = p;
        const char* q = p;
        if (q < e && (*q == '+' || *q == '-')) ++q;
        const char* d0 = q;
        while (q < e && *q >= '0' && *q <= '9') ++q;
        bool dig = q > d0;
        if (q < e && *q == '.') {
            ++q;
            const char* d1 = q;
            while (q < e && *q >= '0' && *q <= '9') ++q;
            dig = dig || q > d1;
        }
        if (dig && q < e && (*q == 'e' || *q == 'E')) {
            const char* r = q + 1;
            if (r < e && (*r == '+' || *r == '-')) ++r;
            const char* d2 = r;
            while (r < e && *r >= '0' && *r <= '9') ++r;
            if (r > d2) q = r;
            else { p = r; v = 0.0f; fail = true; return false; }   // "1e": libstdc++ fails
        }
        if (!dig) { v = 0.0f; fail = true; return false; }
        std::string tok(s, q - s);
        errno = 0;
        char* endp = nullptr;
        float x = std::strtof(tok.c_str(), &endp);
        p = q;
        if (errno == ERANGE && std::isinf(x)) { v = x; fail = true; return false; }
        v = x;
        return true;
    }
    bool num_i(long long& v) {              // operator>>(int)
        if (fail) return false;
        skip();
        const char* q = p;
        if (q < e && (*q == '+' || *q == '-')) ++q;
        const char* d0 = q;
        while (q < e && *q >= '0' && *q <= '9') ++q;
        if (q == d0) { v = 0; fail = true; return false; }
        std::string tok(p, q - p);
        v = std::strtoll(tok.c_str(), nullptr, 10);
        p = q;
        if (v > INT32_MAX || v < INT32_MIN) { fail = true; return false; }
        return true;
    }
};

bool read_file(const char* path, std::string& out) {
    FILE* f = std::fopen(path, "rb");
    if (!f) return false;
    std::fseek(f, 0, SEEK_END);
    long n = std::ftell(f);
    std::fseek(f, 0, SEEK_SET);
    out.resize(n > 0 ? (size_t)n : 0);
    size_t got = n > 0 ? std::fread(&out[0], 1, (size_t)n, f) : 0;
    std::fclose(f);
    out.resize(got);
    return true;
}

// Splits into getline() lines: a trailing newline does not create an extra line that
// matters (an empty line is a no-op for both parsers).
void split_lines(const std::string& t, std::vector<std::pair<const char*, const char*>>& lines) {
    const char* p = t.data();
    const char* e = p + t.size();
    while (p < e) {
        const char* q = (const char*)std::memchr(p, '\n', e - p);
        if (!q) q = e;
        lines.emplace_back(p, q);
        p = q + 1;
    }
}

int load_obj(const char* obj_path, const char* mtl_path, pt_scene& S) {
    std::string mtext, otext;
    if (!read_file(mtl_path, mtext)) { S.err = std::string("Failed to open material file: ") + mtl_path; return PT_E_IO; }
    std::vector<std::pair<const char*, const char*>> L;
    split_lines(mtext, L);
    std::unordered_map<std::string, int> mmap;
    for (size_t li = 0; li < L.size(); li++) {
        if (L[li].second - L[li].first > 127) { S.err = "MTL line longer than 127 chars"; return PT_E_PARSE; }
        Cursor c{L[li].first, L[li].second};
        std::string ident, name;
        c.token(ident);
        c.token(name);
        if (ident != "newmtl") continue;
        float col[4] = {0, 0, 0, 0}, emi[4] = {0, 0, 0, 0}, spc[4] = {0, 0, 0, 0}, dat[4] = {0, 0, 0, 0};
        for (int k = 0; k < 8; k++) {           // exactly 8 property lines (geometry_loader.h:50)
            ++li;
            if (li >= L.size()) break;
            const char* b = L[li].first;
            const char* e = L[li].second;
            if (e - b > 127) { S.err = "MTL line longer than 127 chars"; return PT_E_PARSE; }
            if (e - b < 2) continue;
            Cursor d{b, e};
            std::string thr;
            if (b[0] == 'N' && b[1] == 's') {
                float z = 0;
                d.token(thr);
                d.num_f(z);
                dat[2] = (float)((double)z / 1000.0);
            } else if (b[0] == 'K') {
                float* dst = b[1] == 'e' ? emi : b[1] == 'd' ? col : b[1] == 's' ? spc : nullptr;
                if (dst) {
                    float v[3] = {0, 0, 0};
                    d.token(thr);
                    for (int q = 0; q < 3; q++) d.num_f(v[q]);   // failure -> 0, rest skipped
                    dst[0] = v[0]; dst[1] = v[1]; dst[2] = v[2];
                }
            }
        }
        if (dat[2] > 0) dat[1] = 1.0f;
        dat[0] = 7.5f;
        for (float* q : {col, emi, spc, dat}) S.mats.insert(S.mats.end(), q, q + 4);
        mmap[name] = (int)(S.mats.size() / 16) - 1;
        if (li >= L.size()) break;
    }
    S.n_loaded_mats = (int)(S.mats.size() / 16);

    if (!read_file(obj_path, otext)) { S.err = std::string("Failed to open vertex file: ") + obj_path; return PT_E_IO; }
    L.clear();
    split_lines(otext, L);
    std::vector<float> verts;
    verts.reserve(L.size() * 3);
    std::string cur;
    S.tris.reserve(L.size() * 8);
    for (auto& ln : L) {
        const char* b = ln.first;
        const char* e = ln.second;
        if (e - b > 127) { S.err = "OBJ line longer than 127 chars"; return PT_E_PARSE; }
        if (b == e) continue;
        Cursor c{b, e};
        if (b[0] == 'u') {
            std::string pre, name;
            c.token(pre);
            if (c.token(name)) cur = name;
        } else if (b[0] == 'v') {
            char id;
            float v[3] = {0, 0, 0};
            c.ch(id);
            for (int q = 0; q < 3; q++) c.num_f(v[q]);
            verts.push_back(v[0]); verts.push_back(v[1]); verts.push_back(v[2]);
        } else if (b[0] == 'f') {
            char id;
            long long fi[3] = {0, 0, 0};
            c.ch(id);
            bool ok = c.num_i(fi[0]) && c.num_i(fi[1]) && c.num_i(fi[2]);
            long long nv = (long long)(verts.size() / 3);
            for (int q = 0; q < 3 && ok; q++) ok = fi[q] >= 1 && fi[q] <= nv;
            if (!ok) { S.err = "face index out of range (only `f a b c` with 1-based indices is supported)"; return PT_E_PARSE; }
            auto it = mmap.find(cur);
            int midx = 0;
            if (it == mmap.end()) mmap.emplace(cur, 0);   // reference: mmap[...] inserts 0
            else midx = it->second;
            for (int q = 0; q < 3; q++) {
                const float* v = &verts[3 * (fi[q] - 1)];
                S.tris.insert(S.tris.end(), {v[0], v[1], v[2], 0.0f});
            }
            S.tris.insert(S.tris.end(), {(float)midx, 0.0f, 0.0f, 0.0f});
        }
    }
    return PT_OK;
}

// ---------------------------------------------------------------- robust ingest
// A general Wavefront reader producing the same std140 records.  On files the reference
// parser reads correctly (8-line MTL blocks, `v` / `f a b c` / `usemtl`) it yields the same
// arrays bit for bit (tests/test_scene.py); beyond that it accepts what real exports
// contain -- `f` corners as v, v/vt, v/vt/vn, v//vn, negative (relative) indices, polygons
// (fan-triangulated v0,vi,vi+1), `vt`/`vn`/`vp`/`o`/`g`/`s`/`l`/`p`, comments, `\`
// continuations, any line length, MTL properties in any order and number, `mtllib` -- and
// reports malformed input with the file and line instead of istream's silent zeros.
// Material mapping stays the reference's: Kd -> color, Ke -> emission, Ks -> specular,
// Ns/1000 -> specular probability, smoothness 1 iff that is > 0, emission strength 7.5.
struct Liner {
    std::vector<std::string> lines;
    std::vector<int> line_no;          // 1-based source line of each logical line
    void build(const std::string& text) {
        std::vector<std::pair<const char*, const char*>> L;
        split_lines(text, L);
        std::string acc;
        int start = 0;
        for (size_t i = 0; i < L.size(); i++) {
            std::string ln(L[i].first, L[i].second);
            if (!ln.empty() && ln.back() == '\r') ln.pop_back();
            if (acc.empty()) start = (int)i + 1;
            if (!ln.empty() && ln.back() == '\\') {      // continuation
                ln.pop_back();
                acc += ln;
                acc += ' ';
                continue;
            }
            acc += ln;
            size_t h = acc.find('#');
            if (h != std::string::npos) acc.resize(h);
            lines.push_back(acc);
            line_no.push_back(start);
            acc.clear();
        }
        if (!acc.empty()) { lines.push_back(acc); line_no.push_back(start); }
    }
};

void tokenize(const std::string& s, std::vector<std::string>& out) {
    out.clear();
    size_t i = 0, n = s.size();
    while (i < n) {
        while (i < n && Cursor::ws(s[i])) i++;
        size_t j = i;
        while (j < n && !Cursor::ws(s[j])) j++;
        if (j > i) out.emplace_back(s, i, j - i);
        i = j;
    }
}

bool parse_f(const std::string& t, float& v) {
    if (t.empty()) return false;
    Cursor c{t.data(), t.data() + t.size()};
    if (!c.num_f(v)) return false;
    return c.p == c.e;                    // the whole token is one number
}

// One face corner "v", "v/vt", "v/vt/vn" or "v//vn" -> 0-based vertex index, or -1.
long long corner_index(const std::string& t, long long nv) {
    size_t slash = t.find('/');
    std::string head = t.substr(0, slash);
    if (head.empty()) return -1;
    char* endp = nullptr;
    errno = 0;
    long long k = std::strtoll(head.c_str(), &endp, 10);
    if (*endp != '\0' || errno == ERANGE || k == 0) return -1;
    long long idx = k > 0 ? k - 1 : nv + k;     // negative: relative to the vertices so far
    return (idx >= 0 && idx < nv) ? idx : -1;
}

std::string dir_of(const char* path) {
    std::string p(path);
    size_t s = p.find_last_of('/');
    return s == std::string::npos ? std::string() : p.substr(0, s + 1);
}

int load_mtl_robust(const char* mtl_path, pt_scene& S, std::unordered_map<std::string, int>& mmap) {
    std::string text;
    if (!read_file(mtl_path, text)) { S.err = std::string("Failed to open material file: ") + mtl_path; return PT_E_IO; }
    Liner L;
    L.build(text);
    std::vector<std::string> tk;
    float col[4], emi[4], spc[4], dat[4];
    bool open = false;
    std::string name;
    auto flush = [&]() {
        if (!open) return;
        if (dat[2] > 0) dat[1] = 1.0f;
        dat[0] = 7.5f;
        for (float* q : {col, emi, spc, dat}) S.mats.insert(S.mats.end(), q, q + 4);
        mmap[name] = (int)(S.mats.size() / 16) - 1;
        open = false;
    };
    for (size_t i = 0; i < L.lines.size(); i++) {
        tokenize(L.lines[i], tk);
        if (tk.empty()) continue;
        auto bad = [&](const char* what) {
            S.err = std::string(mtl_path) + ":" + std::to_string(L.line_no[i]) + ": " + what;
            return PT_E_PARSE;
        };
        const std::string& key = tk[0];
        if (key == "newmtl") {
            flush();
            if (tk.size() < 2) return bad("newmtl without a name");
            name = tk[1];
            for (float* q : {col, emi, spc, dat}) q[0] = q[1] = q[2] = q[3] = 0.0f;
            open = true;
        } else if (key == "Kd" || key == "Ks" || key == "Ke") {
            if (!open) return bad("material property before newmtl");
            if (tk.size() < 2) return bad("colour without components");
            if (tk[1] == "spectral" || tk[1] == "xyz") return bad("only rgb colours are supported");
            float v[3];
            if (!parse_f(tk[1], v[0])) return bad("malformed number");
            v[1] = v[2] = v[0];                          // "Kd r" means r r r
            if (tk.size() >= 4) {
                if (!parse_f(tk[2], v[1]) || !parse_f(tk[3], v[2])) return bad("malformed number");
            } else if (tk.size() == 3) {
                return bad("colour with two components");
            }
            float* dst = key == "Kd" ? col : key == "Ke" ? emi : spc;
            dst[0] = v[0]; dst[1] = v[1]; dst[2] = v[2];
        } else if (key == "Ns") {
            if (!open) return bad("material property before newmtl");
            float z;
            if (tk.size() < 2 || !parse_f(tk[1], z)) return bad("malformed number");
            dat[2] = (float)((double)z / 1000.0);
        }
        // Ka, Ni, d, Tr, Tf, illum, map_*, bump, ... carry nothing the shader reads
    }
    flush();
    S.n_loaded_mats = (int)(S.mats.size() / 16);
    return PT_OK;
}

int load_obj_robust(const char* obj_path, const char* mtl_path, pt_scene& S) {
    std::string otext;
    if (!read_file(obj_path, otext)) { S.err = std::string("Failed to open vertex file: ") + obj_path; return PT_E_IO; }
    Liner L;
    L.build(otext);
    std::unordered_map<std::string, int> mmap;
    std::vector<std::string> tk;
    // MTL: the given file, else the OBJ's first `mtllib` (relative to the OBJ's directory)
    std::string mtl = mtl_path ? std::string(mtl_path) : std::string();
    if (mtl.empty()) {
        for (auto& ln : L.lines) {
            tokenize(ln, tk);
            if (tk.size() >= 2 && tk[0] == "mtllib") {
                std::string rest = ln.substr(ln.find("mtllib") + 6);
                size_t a = rest.find_first_not_of(" \t"), b = rest.find_last_not_of(" \t\r");
                mtl = dir_of(obj_path) + rest.substr(a, b - a + 1);
                break;
            }
        }
    }
    if (!mtl.empty()) {
        int rc = load_mtl_robust(mtl.c_str(), S, mmap);
        if (rc) return rc;
    }
    std::vector<float> verts;
    std::vector<long long> poly;
    std::string cur;
    for (size_t i = 0; i < L.lines.size(); i++) {
        tokenize(L.lines[i], tk);
        if (tk.empty()) continue;
        auto bad = [&](const std::string& what) {
            S.err = std::string(obj_path) + ":" + std::to_string(L.line_no[i]) + ": " + what;
            return PT_E_PARSE;
        };
        const std::string& key = tk[0];
        if (key == "v") {
            float v[3];
            if (tk.size() < 4) return bad("vertex with fewer than 3 coordinates");
            for (int q = 0; q < 3; q++)
                if (!parse_f(tk[1 + q], v[q])) return bad("malformed number");
            verts.insert(verts.end(), {v[0], v[1], v[2]});
        } else if (key == "f") {
            const long long nv = (long long)(verts.size() / 3);
            poly.clear();
            for (size_t q = 1; q < tk.size(); q++) {
                long long idx = corner_index(tk[q], nv);
                if (idx < 0) return bad("face corner '" + tk[q] + "' is not a valid vertex reference");
                poly.push_back(idx);
            }
            if (poly.size() < 3) return bad("face with fewer than 3 corners");
            auto it = mmap.find(cur);
            int midx = 0;
            if (it == mmap.end()) mmap.emplace(cur, 0);   // as the reference: unknown -> 0
            else midx = it->second;
            for (size_t q = 1; q + 1 < poly.size(); q++) {
                for (long long c : {poly[0], poly[q], poly[q + 1]}) {
                    const float* v = &verts[3 * c];
                    S.tris.insert(S.tris.end(), {v[0], v[1], v[2], 0.0f});
                }
                S.tris.insert(S.tris.end(), {(float)midx, 0.0f, 0.0f, 0.0f});
            }
        } else if (key == "usemtl") {
            if (tk.size() < 2) return bad("usemtl without a name");
            cur = tk[1];
        }
        // vt, vn, vp, o, g, s, l, p, mtllib, ... carry nothing the shader reads
    }
    return PT_OK;
}

// ---------------------------------------------------------------- BVH
struct Box { float mn[3], mx[3]; };
inline Box empty_box() {
    const float inf = std::numeric_limits<float>::infinity();
    return {{inf, inf, inf}, {-inf, -inf, -inf}};
}
inline void grow(Box& b, const Box& t) {
    for (int a = 0; a < 3; a++) {
        if (t.mn[a] < b.mn[a]) b.mn[a] = t.mn[a];
        if (t.mx[a] > b.mx[a]) b.mx[a] = t.mx[a];
    }
}
// bvh.h:21-27: float extents promoted to double.
inline double area(const Box& b) {
    double x = (float)(b.mx[0] - b.mn[0]);
    double y = (float)(b.mx[1] - b.mn[1]);
    double z = (float)(b.mx[2] - b.mn[2]);
    return 2.0 * (x * y + y * z + x * z);
}

struct TriKey {
    uint32_t w[16];
    bool operator==(const TriKey& o) const { return std::memcmp(w, o.w, sizeof(w)) == 0; }
};
struct TriKeyHash {
    size_t operator()(const TriKey& k) const {
        uint64_t h = 1469598103934665603ull;
        for (int i = 0; i < 16; i++) { h ^= k.w[i]; h *= 1099511628211ull; }
        return (size_t)h;
    }
};

}  // namespace

namespace pt_internal {

// Index of the first triangle equal to each one (all 16 floats, operator== of triangle.h:17-20:
// -0 == +0): the leaf index buildSAHTreeHelper finds with std::find (bvh.h:231-232), by a
// first-occurrence hash map instead of a linear search per leaf.
int first_equal_indices(const float* T, int n, std::vector<int>& out, std::string& err) {
    std::unordered_map<TriKey, int, TriKeyHash> first;
    first.reserve((size_t)n * 2);
    out.resize(n);
    for (int i = 0; i < n; i++) {
        const float* t = T + 16 * (size_t)i;
        TriKey key;
        for (int q = 0; q < 16; q++) {
            if (!std::isfinite(t[q])) { err = "non-finite triangle data"; return PT_E_SCENE; }
            float v = t[q] == 0.0f ? 0.0f : t[q];   // -0 == +0 for operator==
            std::memcpy(&key.w[q], &v, 4);
        }
        out[i] = first.emplace(key, i).first->second;
    }
    return PT_OK;
}

}  // namespace pt_internal

namespace {

struct Builder {
    const float* T;
    int n;
    std::vector<Box> tbox;              // per-triangle bounds
    std::vector<float> cen[3];          // per-axis float centroid sum ((v0+v1)+v2)
    std::vector<int> first_equal;       // index of the first triangle equal to i
    std::vector<float> nodes;           // 12 floats per node
    std::vector<Box> pre, suf;
    std::vector<int> ord[3];

    int node_alloc() {
        size_t k = nodes.size() / 12;
        nodes.resize(nodes.size() + 12, 0.0f);
        return (int)k;
    }

    // find_split (bvh.h:173-218) on `idx` (the node's vector order); returns the split
    // position and leaves the chosen order in `idx`.
    size_t split(std::vector<int>& idx, const Box& overall) {
        size_t m = idx.size();
        double SA = area(overall);
        double best = std::numeric_limits<double>::infinity();
        int best_axis = -1;
        size_t best_split = 0;
        pre.resize(m);
        suf.resize(m);
        const std::vector<int>* prev = &idx;
        for (int a = 0; a < 3; a++) {
            std::vector<int>& o = ord[a];
            o.assign(prev->begin(), prev->end());
            const float* c = cen[a].data();
            std::stable_sort(o.begin(), o.end(), [c](int i, int j) { return c[i] < c[j]; });
            prev = &o;
            Box run = empty_box();
            for (size_t i = 0; i < m; i++) { grow(run, tbox[o[i]]); pre[i] = run; }
            run = empty_box();
            for (size_t i = m; i-- > 0;) { grow(run, tbox[o[i]]); suf[i] = run; }
            for (int s = 1; (size_t)s < m; s += (int)(m / 60 + 1)) {
                double SA1 = area(pre[s - 1]), SA2 = area(suf[s]);
                double cost = 1.0 + (SA1 / SA) * s * 1.0 + (SA2 / SA) * (double)(m - s) * 1.0;
                if (cost < best) { best = cost; best_axis = a; best_split = (size_t)s; }
            }
        }
        if (best_axis < 0) {            // degenerate (SA == 0): median of the z order
            idx.assign(ord[2].begin(), ord[2].end());
            return m / 2;
        }
        idx.assign(ord[best_axis].begin(), ord[best_axis].end());
        return best_split;
    }

    int run(float* out, int max_nodes, int* n_nodes, std::string& err) {
        tbox.resize(n);
        for (int a = 0; a < 3; a++) cen[a].resize(n);
        int rc = pt_internal::first_equal_indices(T, n, first_equal, err);
        if (rc) return rc;
        for (int i = 0; i < n; i++) {
            const float* t = T + 16 * (size_t)i;
            Box b = empty_box();
            for (int vtx = 0; vtx < 3; vtx++)
                for (int a = 0; a < 3; a++) {
                    float c = t[4 * vtx + a];
                    if (c < b.mn[a]) b.mn[a] = c;
                    if (c > b.mx[a]) b.mx[a] = c;
                }
            tbox[i] = b;
            for (int a = 0; a < 3; a++) cen[a][i] = (t[a] + t[4 + a]) + t[8 + a];
        }
        nodes.reserve((size_t)24 * n);
        node_alloc();
        struct Item { int node; std::vector<int> idx; };
        std::vector<Item> stack;
        {
            Item root{0, std::vector<int>(n)};
            for (int i = 0; i < n; i++) root.idx[i] = i;
            stack.push_back(std::move(root));
        }
        while (!stack.empty()) {
            Item it = std::move(stack.back());
            stack.pop_back();
            Box ov = empty_box();
            for (int i : it.idx) grow(ov, tbox[i]);
            float* nd = &nodes[12 * (size_t)it.node];
            const float inf = std::numeric_limits<float>::infinity();
            nd[0] = ov.mn[0]; nd[1] = ov.mn[1]; nd[2] = ov.mn[2]; nd[3] = inf;
            nd[4] = ov.mx[0]; nd[5] = ov.mx[1]; nd[6] = ov.mx[2]; nd[7] = -inf;
            if (it.idx.size() <= 2) {
                nd[8] = (float)first_equal[it.idx.front()];
                nd[9] = (float)first_equal[it.idx.back()];
                nd[10] = -1.0f;
                nd[11] = -1.0f;
                continue;
            }
            size_t s = split(it.idx, ov);
            int l = node_alloc();
            int r = node_alloc();
            nd = &nodes[12 * (size_t)it.node];
            nd[8] = -1.0f; nd[9] = -1.0f;
            nd[10] = (float)l; nd[11] = (float)r;
            Item L{l, std::vector<int>(it.idx.begin(), it.idx.begin() + s)};
            Item R{r, std::vector<int>(it.idx.begin() + s, it.idx.end())};
            std::vector<int>().swap(it.idx);
            stack.push_back(std::move(R));
            stack.push_back(std::move(L));
        }
        // build_links (bvh.h:84-98), iteratively.  Reads the pre-link child fields.
        size_t nn = nodes.size() / 12;
        std::vector<float> links(nn * 2);
        std::vector<std::pair<int, int>> st;
        st.emplace_back(0, -1);
        while (!st.empty()) {
            auto [cur, next_right] = st.back();
            st.pop_back();
            const float* nd = &nodes[12 * (size_t)cur];
            if (nd[11] > -1.0f) {
                int c1 = (int)nd[10], c2 = (int)nd[11];
                links[2 * cur] = (float)c1;
                links[2 * cur + 1] = (float)next_right;
                st.emplace_back(c2, next_right);
                st.emplace_back(c1, c2);
            } else {
                links[2 * cur] = (float)next_right;
                links[2 * cur + 1] = (float)next_right;
            }
        }
        for (size_t i = 0; i < nn; i++) {
            nodes[12 * i + 10] = links[2 * i];
            nodes[12 * i + 11] = links[2 * i + 1];
        }
        *n_nodes = (int)nn;
        if (out) {
            if ((int)nn > max_nodes) { err = "node buffer too small"; return PT_E_ARG; }
            std::memcpy(out, nodes.data(), nodes.size() * sizeof(float));
        }
        return PT_OK;
    }
};

thread_local std::string g_bvh_err;

}  // namespace

namespace pt_internal {
void set_bvh_error(const std::string& msg) { g_bvh_err = msg; }
}

namespace {

// The structure the culling walk relies on, on the std140 records: from
// the root, a full binary tree threaded in preorder -- an internal node's hit link is its
// left child L, L's miss link its right child R, R's miss link the node's own -- in which
// every internal box contains both children's boxes (exact float compares).  A walk that
// enters a subtree the exact test would skip then leaves it at the same miss link, and any
// leaf inside has a box within the skipped one, which fails the exact test too.
// A link field as a node index: finite, integral and in [-1, n_nodes), else -2 (never a
// valid link; casting NaN or a huge float to int would be undefined behaviour).
static int link_of(float v, int n_nodes) {
    if (!(v >= -1.0f && v < (float)n_nodes) || v != (float)(int)v) return -2;
    return (int)v;
}

static bool nested_tree(const float* bvh, int n_nodes) {
    if (n_nodes <= 0) return false;
    std::vector<unsigned char> seen(n_nodes, 0);
    std::vector<std::pair<int, int>> st;   // (node, the miss link it must carry)
    st.emplace_back(0, -1);
    while (!st.empty()) {
        const int x = st.back().first, after = st.back().second;
        st.pop_back();
        if (x < 0 || x >= n_nodes || seen[x]) return false;
        seen[x] = 1;
        const float* nd = bvh + 12 * (size_t)x;
        const int hit = link_of(nd[10], n_nodes), miss = link_of(nd[11], n_nodes);
        if (hit == -2 || miss != after) return false;
        if (nd[8] > -1.0f) {                       // leaf: its hit link is its miss link
            if (hit != miss) return false;
            continue;
        }
        const int l = hit;
        if (l < 0) return false;
        const int r = link_of(bvh[12 * (size_t)l + 11], n_nodes);
        if (r < 0 || r == after) return false;
        for (int ch : {l, r}) {
            const float* cb = bvh + 12 * (size_t)ch;
            for (int q = 0; q < 3; q++)
                if (!(nd[q] <= cb[q] && cb[4 + q] <= nd[4 + q])) return false;
        }
        st.emplace_back(r, after);
        st.emplace_back(l, r);
    }
    return true;
}

}  // namespace

extern "C" {

const char* pt_bvh_last_error(void) { return g_bvh_err.c_str(); }

int pt_scene_build_bvh_gpu(pt_scene* s, int device) {
    if (!s) return PT_E_ARG;
    const int nt = (int)(s->tris.size() / 16);
    if (nt <= 0) { s->err = "scene has no triangles (the reference indexes triangles[0])"; return PT_E_SCENE; }
    int nn = 0;
    std::vector<float> nodes(12 * (2 * (size_t)nt - 1));
    const int rc = pt_bvh_build_gpu(s->tris.data(), nt, nodes.data(), 2 * nt - 1, &nn, device);
    if (rc) { s->err = g_bvh_err; return rc; }
    nodes.resize(12 * (size_t)nn);
    s->nodes.swap(nodes);
    return PT_OK;
}

int pt_bvh_build(const float* tris, int n_tris, float* nodes_out, int max_nodes, int* n_nodes) {
    if (!tris || n_tris <= 0 || !n_nodes) { g_bvh_err = "empty triangle list"; return PT_E_ARG; }
    if (n_tris > (1 << 23)) { g_bvh_err = "more than 2^23 triangles (float index limit)"; return PT_E_SCENE; }
    Builder b;
    b.T = tris;
    b.n = n_tris;
    return b.run(nodes_out, max_nodes, n_nodes, g_bvh_err);
}

int pt_scene_load_obj(const char* obj_path, const char* mtl_path, pt_scene** out) {
    if (!obj_path || !mtl_path || !out) return PT_E_ARG;
    pt_scene* s = new pt_scene();
    int rc = load_obj(obj_path, mtl_path, *s);
    *out = s;   // returned even on error so pt_scene_last_error() can explain
    return rc;
}

int pt_scene_load_obj_ex(const char* obj_path, const char* mtl_path, int flags, pt_scene** out) {
    if (!out) return PT_E_ARG;
    *out = nullptr;
    if (!obj_path) return PT_E_ARG;
    if (flags & ~PT_LOAD_ROBUST) return PT_E_ARG;
    if (!(flags & PT_LOAD_ROBUST)) return pt_scene_load_obj(obj_path, mtl_path, out);
    pt_scene* s = new pt_scene();
    int rc = load_obj_robust(obj_path, mtl_path, *s);
    *out = s;
    return rc;
}

int pt_scene_from_arrays(const float* tris, int n_tris, const float* mats, int n_mats, pt_scene** out) {
    if (!out || n_tris < 0 || n_mats < 0 || (n_tris && !tris) || (n_mats && !mats)) return PT_E_ARG;
    pt_scene* s = new pt_scene();
    s->tris.assign(tris, tris + 16 * (size_t)n_tris);
    s->mats.assign(mats, mats + 16 * (size_t)n_mats);
    s->n_loaded_mats = n_mats;
    *out = s;
    return PT_OK;
}

int pt_scene_add_builtins(pt_scene* s) {
    if (!s) return PT_E_ARG;
    if (s->builtins) return PT_OK;
    // ogl_path_trace.h:415-444: light, spec, diffuse, ground, metal (w lanes as written).
    static const float M[5][16] = {
        {0, 0, 0, 1, 0.99f, 0.95f, 0.78f, 1, 0, 0, 0, 0, 1.5f, 0, 0, 0},
        {1, 0.39f, 0.28f, 1, 0, 0, 0, 1, 1, 1, 1, 1, 0, 1, 0.18f, 0},
        {1, 0.5f, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 0, 1, 0.1f, 0},
        {1, 0.9f, 0.9f, 1, 0, 0, 0, 1, 0, 0, 0, 1, 0, 0, 0, 0},
        {0.9f, 0.9f, 0.1f, 1, 0, 0, 0, 1, 1, 1, 1, 1, 0, 0.9f, 0.91f, 0},
    };
    int m = s->n_loaded_mats;
    s->mats.resize(16 * (size_t)m);
    s->mats.insert(s->mats.end(), &M[0][0], &M[0][0] + 80);
    // ogl_path_trace.h:498-501: s3 = metal sphere, the only one uploaded.
    const float sp[8] = {-0.5f, 3.0f, 1.0f, 0.8f, (float)m + 4.0f, 0, 0, 0};
    s->spheres.assign(sp, sp + 8);
    s->builtins = true;
    return PT_OK;
}

int pt_scene_build_bvh(pt_scene* s) {
    if (!s) return PT_E_ARG;
    int nt = (int)(s->tris.size() / 16);
    if (nt <= 0) { s->err = "scene has no triangles (the reference indexes triangles[0])"; return PT_E_SCENE; }
    Builder b;
    b.T = s->tris.data();
    b.n = nt;
    int nn = 0;
    int rc = b.run(nullptr, 0, &nn, s->err);
    if (rc) return rc;
    s->nodes.swap(b.nodes);
    return PT_OK;
}

int pt_scene_counts(const pt_scene* s, int c[5]) {
    if (!s || !c) return PT_E_ARG;
    c[0] = (int)(s->tris.size() / 16);
    c[1] = (int)(s->mats.size() / 16);
    c[2] = (int)(s->spheres.size() / 8);
    c[3] = (int)(s->nodes.size() / 12);
    c[4] = s->n_loaded_mats;
    return PT_OK;
}

static int copy_out(const std::vector<float>& v, int per, float* dst, int max) {
    if (!dst) return PT_E_ARG;
    if ((size_t)max * per < v.size()) return PT_E_ARG;
    std::memcpy(dst, v.data(), v.size() * sizeof(float));
    return PT_OK;
}
int pt_scene_get_tris(const pt_scene* s, float* d, int m) { return s ? copy_out(s->tris, 16, d, m) : PT_E_ARG; }
int pt_scene_get_mats(const pt_scene* s, float* d, int m) { return s ? copy_out(s->mats, 16, d, m) : PT_E_ARG; }
int pt_scene_get_spheres(const pt_scene* s, float* d, int m) { return s ? copy_out(s->spheres, 8, d, m) : PT_E_ARG; }
int pt_scene_get_nodes(const pt_scene* s, float* d, int m) { return s ? copy_out(s->nodes, 12, d, m) : PT_E_ARG; }

const char* pt_scene_last_error(const pt_scene* s) { return s ? s->err.c_str() : g_bvh_err.c_str(); }
void pt_scene_free(pt_scene* s) { delete s; }

void pt_aces_rgba8_host(const float* rgba, long long n, unsigned char* out) {
    for (long long i = 0; i < n; i++) {
        for (int c = 0; c < 3; c++) {
            float v = rgba[4 * i + c];
            float tm = (v * (2.51f * v + 0.03f)) / (v * (2.43f * v + 0.59f) + 0.14f);
            tm = tm < 0.0f ? 0.0f : (tm > 1.0f ? 1.0f : tm);
            if (!(tm == tm)) tm = 0.0f;
            out[4 * i + c] = (unsigned char)(int)(tm * 255.0f + 0.5f);
        }
        out[4 * i + 3] = 255;
    }
}

int pt_bvh_culling_ok(const float* nodes, int n_nodes) {
    return nodes && n_nodes > 0 && nested_tree(nodes, n_nodes) ? 1 : 0;
}

}  // extern "C"
