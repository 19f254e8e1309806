// pt_obj.cpp — native OBJ ingest and Mesh host operations.
//
// pt_obj_load restates OBJ.Load (OBJ.cs:11-165) including its quirks, so a mesh
// loaded here is the Triangle[] the C# loader builds:
//   - each line is lower-cased and split on ' ' only (empty words dropped); a tab
//     is part of a word, so "v\t1 2 3" is an unknown keyword (OBJ.cs:33-35);
//   - the normal list starts with a dummy (0,0,0) (OBJ.cs:18), and face indices are
//     `index - 1` into it: "vn" k resolves to file normal k-1, "vn" 1 to the dummy;
//   - a face vertex is split on "//" and "/" with empty parts removed
//     (OBJ.cs:89-93), so "v//n" reads n as a texture index and keeps normal 0
//     (the dummy);
//   - faces are fan-triangulated (0, i, i+1) (OBJ.cs:110-113); missing texture /
//     normal indices are 0; Triangle.FixNormals replaces zero normals by the face
//     normal (Triangle.cs:199-204, 224-237);
//   - mtllib resolves `cwd + "\\" + name` and usemtl only ever finds copies of the
//     parent material (Material is a struct: LoadMTL's edits never reach matList,
//     OBJ.cs:167-219), so every triangle keeps the caller's material.
// Numbers parse as float.Parse does under the invariant culture (strtof, round to
// nearest).  A malformed number or an out-of-range index fails the whole load, as
// the C# exception would.
#include <cerrno>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <unordered_map>
#include <vector>

#include "../../include/ptsharp_hip.h"

// Built with -ffp-contract=off (Makefile): the face normal is FixNormals' fp32 sequence, unfused.

namespace {

struct F3 {
    float x, y, z;
};

thread_local std::string g_obj_error;

int obj_fail(const std::string& m) {
    g_obj_error = m;
    return PT_ERR_INVALID_ARG;
}

// float.Parse / int.Parse (invariant culture) allow surrounding white space.
// A word of a line: [p, p + n) (no allocation; lines are parsed in place).
struct Word {
    const char* p;
    size_t n;
    bool eq(const char* lit) const { return std::strlen(lit) == n && std::memcmp(p, lit, n) == 0; }
};

Word trim(Word w) {
    auto ws = [](char c) { return c == ' ' || c == '\t' || c == '\n' || c == '\v' || c == '\f' || c == '\r'; };
    while (w.n && ws(w.p[0])) { w.p++; w.n--; }
    while (w.n && ws(w.p[w.n - 1])) w.n--;
    return w;
}

// strtof / strtol need a terminated string: words are copied to a stack buffer (a longer word,
// which no number is, goes through a std::string).
template <class T, class F>
bool parse_num(Word w, T& out, F conv) {
    w = trim(w);
    if (!w.n) return false;
    char buf[64];
    std::string big;
    const char* s = buf;
    if (w.n < sizeof buf) { std::memcpy(buf, w.p, w.n); buf[w.n] = 0; }
    else { big.assign(w.p, w.n); s = big.c_str(); }
    char* end = nullptr;
    out = conv(s, &end);
    return end == s + w.n;
}
bool parse_float(Word w, float& out) {
    return parse_num(w, out, [](const char* s, char** e) { return std::strtof(s, e); });
}
bool parse_int(Word w, long& out) {
    return parse_num(w, out, [](const char* s, char** e) { return std::strtol(s, e, 10); });
}

// Vector.Sub / Cross / Normalize in fp32 (Vector.cs; pt_math.h has the same ops).
F3 sub(F3 a, F3 b) { return F3{a.x - b.x, a.y - b.y, a.z - b.z}; }
F3 cross(F3 a, F3 b) { return F3{a.y * b.z - a.z * b.y, a.z * b.x - a.x * b.z, a.x * b.y - a.y * b.x}; }
F3 normalize(F3 a) {
    float len = std::sqrt((a.x * a.x + a.y * a.y) + a.z * a.z);
    return F3{a.x / len, a.y / len, a.z / len};
}
bool is_zero(F3 a) { return a.x == 0.f && a.y == 0.f && a.z == 0.f; }

// String.Split(new[] {"//", "/"}, RemoveEmptyEntries): at most `max` parts kept (the rest are unused)
size_t split_slashes(Word s, Word* out, size_t max) {
    size_t k = 0, start = 0;
    for (size_t i = 0; i <= s.n;) {
        if (i == s.n || s.p[i] == '/') {
            if (i > start && k < max) out[k] = Word{s.p + start, i - start};
            if (i > start) k++;
            if (i == s.n) break;
            i += (i + 1 < s.n && s.p[i + 1] == '/') ? 2 : 1;
            start = i;
        } else {
            i++;
        }
    }
    return k;
}

struct Loader {
    std::vector<F3> vs, vts, vns{F3{0.f, 0.f, 0.f}};
    std::vector<float> v1, v2, v3, n1, n2, n3, t1, t2, t3;
    std::vector<Word> words;             // reused per line
    std::vector<long> fv, ft, fn;

    template <class Vec>
    bool at(const Vec& list, long idx, F3& out) const {
        if (idx < 0 || (size_t)idx >= list.size()) return false;
        out = list[(size_t)idx];
        return true;
    }
    static void put(std::vector<float>& a, F3 v) {
        a.push_back(v.x);
        a.push_back(v.y);
        a.push_back(v.z);
    }

    // One line, lower-cased in place (ToLower is invariant for ASCII), split on ' ' (OBJ.cs:33-35).
    int line(char* ln, size_t len, size_t lineno) {
        for (size_t i = 0; i < len; i++) ln[i] = (char)std::tolower((unsigned char)ln[i]);
        words.clear();
        size_t start = 0;
        for (size_t i = 0; i <= len; i++) {
            if (i == len || ln[i] == ' ') {
                if (i > start) words.push_back(Word{ln + start, i - start});
                start = i + 1;
            }
        }
        if (words.empty()) return PT_OK;
        const Word type = words[0];
        const Word* w = words.data() + 1;
        const size_t nw = words.size() - 1;
        auto where = [&]() { return " (line " + std::to_string(lineno) + ")"; };
        if (type.eq("v") || type.eq("vn")) {
            F3 v;
            if (nw < 3 || !parse_float(w[0], v.x) || !parse_float(w[1], v.y) || !parse_float(w[2], v.z))
                return obj_fail("bad " + std::string(type.p, type.n) + where());
            (type.eq("v") ? vs : vns).push_back(v);
        } else if (type.eq("vt")) {
            F3 v{0.f, 0.f, 0.f};
            if (nw < 2 || !parse_float(w[0], v.x) || !parse_float(w[1], v.y))
                return obj_fail("bad vt" + where());
            vts.push_back(v);
        } else if (type.eq("f")) {
            const size_t n = nw;
            fv.assign(n, 0); ft.assign(n, 0); fn.assign(n, 0);
            for (size_t count = 0; count < n; count++) {
                Word p[3];
                const size_t np = split_slashes(w[count], p, 3);
                long x;
                if (np > 0) { if (!parse_int(p[0], x)) return obj_fail("bad face index" + where()); fv[count] = x - 1; }
                if (np > 1) { if (!parse_int(p[1], x)) return obj_fail("bad face index" + where()); ft[count] = x - 1; }
                if (np > 2) { if (!parse_int(p[2], x)) return obj_fail("bad face index" + where()); fn[count] = x - 1; }
            }
            for (size_t i = 1; i + 1 < n; i++) {
                const size_t c[3] = {0, i, i + 1};
                F3 V[3], T[3], N[3];
                for (int k = 0; k < 3; k++) {
                    V[k] = T[k] = F3{0.f, 0.f, 0.f};
                    if (!vs.empty() && !at(vs, fv[c[k]], V[k])) return obj_fail("vertex index out of range" + where());
                    if (!vts.empty() && !at(vts, ft[c[k]], T[k])) return obj_fail("texture index out of range" + where());
                    if (!at(vns, fn[c[k]], N[k])) return obj_fail("normal index out of range" + where());
                }
                // Triangle.FixNormals
                const F3 face = normalize(cross(sub(V[1], V[0]), sub(V[2], V[0])));
                for (int k = 0; k < 3; k++)
                    if (is_zero(N[k])) N[k] = face;
                put(v1, V[0]); put(v2, V[1]); put(v3, V[2]);
                put(n1, N[0]); put(n2, N[1]); put(n3, N[2]);
                put(t1, T[0]); put(t2, T[1]); put(t3, T[2]);
            }
        }
        // mtllib / usemtl: no effect on the result (see the header); other keywords ignored
        return PT_OK;
    }
};

float* copy_out(const std::vector<float>& a) {
    float* p = (float*)std::malloc(a.empty() ? sizeof(float) : a.size() * sizeof(float));
    if (p && !a.empty()) std::memcpy(p, a.data(), a.size() * sizeof(float));
    return p;
}

struct KeyHash {
    size_t operator()(const F3& k) const {
        uint32_t b[3];
        std::memcpy(b, &k, sizeof b);
        uint64_t h = 0x9E3779B97F4A7C15ull;
        for (uint32_t x : b) h = (h ^ x) * 0xBF58476D1CE4E5B9ull;
        return (size_t)(h ^ (h >> 31));
    }
};
struct KeyEq {
    bool operator()(const F3& a, const F3& b) const { return a.x == b.x && a.y == b.y && a.z == b.z; }
};

}  // namespace

extern "C" {

const char* pt_obj_last_error(void) { return g_obj_error.c_str(); }

int pt_obj_load(const char* path, pt_mesh_data* out) {
    if (!path || !out) return obj_fail("NULL argument");
    std::memset(out, 0, sizeof *out);
    FILE* f = std::fopen(path, "rb");
    if (!f) return obj_fail(std::string("Unable to open \"") + path + "\", does not exist.");
    Loader L;
    std::string ln;
    size_t lineno = 0;
    int rc = PT_OK;
    // StreamReader.ReadLine: "\n", "\r\n" and "\r" end a line.  The file is read in 1-MB blocks.
    std::vector<char> blk(1u << 20);
    bool cr = false;   // the previous block ended on '\r': a '\n' starting this one belongs to it
    for (;;) {
        const size_t got = std::fread(blk.data(), 1, blk.size(), f);
        size_t i = 0;
        if (cr && got > 0 && blk[0] == '\n') i = 1;
        cr = false;
        for (; i < got && rc == PT_OK; i++) {
            const char ch = blk[i];
            if (ch == '\n' || ch == '\r') {
                rc = L.line(ln.data(), ln.size(), ++lineno);
                ln.clear();
                if (ch == '\r') {
                    if (i + 1 < got) { if (blk[i + 1] == '\n') i++; }
                    else cr = true;
                }
            } else {
                // the run up to the next line end in one append
                size_t j = i;
                while (j < got && blk[j] != '\n' && blk[j] != '\r') j++;
                ln.append(blk.data() + i, j - i);
                i = j - 1;
            }
        }
        if (rc != PT_OK || got < blk.size()) break;
    }
    if (rc == PT_OK && std::ferror(f)) rc = obj_fail(std::string("read error on \"") + path + "\"");
    if (rc == PT_OK && !ln.empty()) rc = L.line(ln.data(), ln.size(), ++lineno);
    std::fclose(f);
    if (rc != PT_OK) return rc;
    const size_t n = L.v1.size() / 3;
    if (n > 0x7FFFFFFF) return obj_fail("too many triangles");
    out->num_triangles = (int32_t)n;
    float** dst[9] = {&out->v1, &out->v2, &out->v3, &out->n1, &out->n2, &out->n3, &out->t1, &out->t2, &out->t3};
    const std::vector<float>* src[9] = {&L.v1, &L.v2, &L.v3, &L.n1, &L.n2, &L.n3, &L.t1, &L.t2, &L.t3};
    for (int k = 0; k < 9; k++) {
        *dst[k] = copy_out(*src[k]);
        if (!*dst[k]) {
            pt_mesh_free(out);
            return obj_fail("out of host memory");
        }
    }
    return PT_OK;
}

void pt_mesh_free(pt_mesh_data* m) {
    if (!m) return;
    float** p[9] = {&m->v1, &m->v2, &m->v3, &m->n1, &m->n2, &m->n3, &m->t1, &m->t2, &m->t3};
    for (auto q : p) {
        std::free(*q);
        *q = nullptr;
    }
    m->num_triangles = 0;
}

// Mesh.SmoothNormals (Mesh.cs:191-229): per distinct vertex position, the fp32 sum
// of its corner normals in triangle order (V1, V2, V3 of each triangle), then
// Normalize; every corner takes its position's normal.  Vertices compare as
// Vector ==, so -0 and +0 are one key.
int pt_mesh_smooth_normals(int32_t n, const float* v1, const float* v2, const float* v3, float* n1, float* n2,
                           float* n3) {
    if (n < 0 || (n > 0 && (!v1 || !v2 || !v3 || !n1 || !n2 || !n3))) return obj_fail("bad mesh arrays");
    const float* V[3] = {v1, v2, v3};
    float* N[3] = {n1, n2, n3};
    auto key = [&](int k, int32_t i) {
        const float* p = V[k] + 3 * (size_t)i;
        return F3{p[0] + 0.f, p[1] + 0.f, p[2] + 0.f};  // -0 → +0
    };
    std::unordered_map<F3, F3, KeyHash, KeyEq> acc;
    acc.reserve((size_t)n * 2 + 1);
    for (int32_t i = 0; i < n; i++)
        for (int k = 0; k < 3; k++) {
            F3& a = acc.emplace(key(k, i), F3{0.f, 0.f, 0.f}).first->second;
            const float* q = N[k] + 3 * (size_t)i;
            a = F3{a.x + q[0], a.y + q[1], a.z + q[2]};
        }
    for (auto& kv : acc) kv.second = normalize(kv.second);
    for (int32_t i = 0; i < n; i++)
        for (int k = 0; k < 3; k++) {
            auto it = acc.find(key(k, i));
            if (it == acc.end()) return obj_fail("NaN vertex: no SmoothNormals entry (the reference throws)");
            const F3 s = it->second;
            float* q = N[k] + 3 * (size_t)i;
            q[0] = s.x; q[1] = s.y; q[2] = s.z;
        }
    return PT_OK;
}

}  // extern "C"
