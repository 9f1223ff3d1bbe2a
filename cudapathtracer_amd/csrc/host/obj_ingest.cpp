// obj_ingest.cpp -- OBJ/MTL reader reproducing tinyobjloader 0.9.13 as vendored by the
// reference (tiny_obj_loader.cc:8), restated for the fields loadOBJ consumes.
//
// Behaviour kept on purpose (each is observable in the arrays loadOBJ builds):
//  * numbers go through the greedy decimal scanner of tryParseDouble (.cc:127-241): digits
//    are accumulated in double with pow(10,-k) per fractional digit, then
//    ldexp(m * pow(5,e), e); a token that does not start with a sign or digit (".5") is 0;
//  * faces are fan-triangulated (v0, v[k-1], v[k]) and vertices are de-duplicated per shape
//    on the (v, vt, vn) index triple in first-use order (.cc:304-339, 361-411);
//  * a shape is emitted at every `usemtl`, `g`, `o` and at EOF when faces are pending, with
//    the material in force for those faces (.cc:764-792, 812-878);
//  * `mtllib` reads <basepath><name>; tinyobj's reader always appends a final material
//    (a default one named "" for an empty or missing file) and a missing file aborts the OBJ
//    read at that line, returning the shapes emitted so far (.cc:594-636, 794-810);
//  * lines are read up to 8191 characters, trailing '\r' trimmed, leading blanks skipped,
//    '#' lines ignored (.cc:682-708).
#include <cctype>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <map>
#include <sstream>
#include <tuple>
#include <unordered_map>

#include "host_internal.h"

namespace pt {

namespace {

constexpr size_t kMaxLine = 8191;   // std::istream::getline(buf, 8192)

inline bool blank(char c) { return c == ' ' || c == '\t'; }
inline bool line_end(char c) { return c == '\r' || c == '\n' || c == '\0'; }
inline bool digit(char c) { return c >= '0' && c <= '9'; }

// Visit the logical lines tinyobj's getline loop would see, in place: each line is
// NUL-terminated inside `text` (an embedded NUL ends the line early, as getline's C string
// does); a line longer than kMaxLine is cut there and is the last line read (failbit).
template <typename F>
void for_each_line(std::string& text, F&& visit)
{
    size_t pos = 0;
    const size_t n = text.size();
    char* base = &text[0];
    while (pos < n) {
        const char* nl = static_cast<const char*>(memchr(base + pos, '\n', n - pos));
        const size_t stop = nl ? static_cast<size_t>(nl - base) : n;
        if (stop - pos > kMaxLine) {
            base[pos + kMaxLine] = '\0';
            visit(base + pos);
            return;
        }
        if (stop < n) base[stop] = '\0';
        visit(base + pos);
        pos = nl ? stop + 1 : n;
    }
}

bool slurp(const std::string& path, std::string* out)
{
    std::ifstream f(path.c_str(), std::ios::in | std::ios::binary);
    if (!f) return false;
    std::ostringstream ss;
    ss << f.rdbuf();
    *out = ss.str();
    return true;
}

// Returns a pointer to the first non-blank char of a trimmed line, or nullptr to skip it.
const char* line_start(char* line)
{
    size_t len = strlen(line);
    if (len > 0 && line[len - 1] == '\r') line[--len] = '\0';
    if (len == 0) return nullptr;
    const char* t = line;
    t += strspn(t, " \t");
    if (*t == '\0' || *t == '#') return nullptr;
    return t;
}

float next_real(const char*& tok)
{
    tok += strspn(tok, " \t");
    const char* end = tok + strcspn(tok, " \t\r");
    double v = 0.0;
    parse_real(tok, end, &v);
    tok = end;
    return static_cast<float>(v);
}

// Index word "i", "i/j", "i//k", "i/j/k" -> zero-based triple; -1 = absent (.cc:271-302).
struct VIdx { int v, vt, vn; };

inline int rebase(int idx, int count)
{
    if (idx > 0) return idx - 1;
    if (idx == 0) return 0;
    return count + idx;
}

VIdx next_vidx(const char*& tok, int nv, int nvn, int nvt)
{
    VIdx r{-1, -1, -1};
    r.v = rebase(atoi(tok), nv);
    tok += strcspn(tok, "/ \t\r");
    if (*tok != '/') return r;
    ++tok;
    if (*tok == '/') {
        ++tok;
        r.vn = rebase(atoi(tok), nvn);
        tok += strcspn(tok, "/ \t\r");
        return r;
    }
    r.vt = rebase(atoi(tok), nvt);
    tok += strcspn(tok, "/ \t\r");
    if (*tok != '/') return r;
    ++tok;
    r.vn = rebase(atoi(tok), nvn);
    tok += strcspn(tok, "/ \t\r");
    return r;
}

std::string first_word(const char* t)
{
    char buf[4096];
    buf[0] = '\0';
    if (sscanf(t, "%4095s", buf) != 1) return std::string();
    return std::string(buf);
}

// Material library reader (.cc:413-615).  Returns true when the file opened.
bool read_mtl(const std::string& path, std::vector<ObjMaterial>& mats, std::map<std::string, int>& by_name)
{
    std::string text;
    const bool opened = slurp(path, &text);
    ObjMaterial cur;
    auto reset = [&cur]() {
        cur.name.clear();
        for (int i = 0; i < 3; ++i) { cur.diffuse[i] = 0.f; cur.emission[i] = 0.f; }
    };
    auto commit = [&]() {
        by_name.insert(std::make_pair(cur.name, static_cast<int>(mats.size())));
        mats.push_back(cur);
    };
    reset();
    if (opened) {
        for_each_line(text, [&](char* line) {
            const char* t = line_start(line);
            if (!t) return;
            if (strncmp(t, "newmtl", 6) == 0 && blank(t[6])) {
                if (!cur.name.empty()) commit();
                reset();
                cur.name = first_word(t + 7);
                return;
            }
            if (t[0] == 'K' && (t[1] == 'd' || t[1] == 'e') && blank(t[2])) {
                float* dst = (t[1] == 'd') ? cur.diffuse : cur.emission;
                t += 2;
                float r = next_real(t);
                float g = next_real(t);
                float b = next_real(t);
                dst[0] = r; dst[1] = g; dst[2] = b;
                return;
            }
            // Ka/Ks/Kt/Ni/Ns/illum/d/Tr/map_*/unknown keys do not reach loadOBJ.
        });
    }
    commit();   // tinyobj always flushes the last (possibly default, unnamed) material
    return opened;
}

// exportFaceGroupToShape (.cc:361-411) with a fresh vertex cache per shape.
struct VIdxHash {
    size_t operator()(const std::tuple<int, int, int>& k) const
    {
        uint64_t h = static_cast<uint32_t>(std::get<0>(k));
        h = h * 0x9E3779B97F4A7C15ull ^ static_cast<uint32_t>(std::get<1>(k));
        h = h * 0x9E3779B97F4A7C15ull ^ static_cast<uint32_t>(std::get<2>(k));
        return static_cast<size_t>(h ^ (h >> 29));
    }
};

// Faces are stored flat: face f has the index words fv[fstart[f] .. fstart[f+1]).
bool emit_shape(const std::vector<VIdx>& fv, const std::vector<uint32_t>& fstart, const std::vector<float>& v,
                int material, const std::string& name, std::vector<ObjShape>& shapes, std::string* err)
{
    if (fstart.size() < 2) return true;
    ObjShape sh;
    std::unordered_map<std::tuple<int, int, int>, uint32_t, VIdxHash> seen;
    seen.reserve(fv.size());
    auto vertex = [&](const VIdx& k, uint32_t* out) -> bool {
        auto key = std::make_tuple(k.v, k.vn, k.vt);
        auto it = seen.find(key);
        if (it != seen.end()) { *out = it->second; return true; }
        if (k.v < 0 || static_cast<size_t>(3 * k.v + 2) >= v.size()) {
            *err = "face references vertex " + std::to_string(k.v + 1) + " which does not exist";
            return false;
        }
        sh.positions.push_back(v[3 * k.v + 0]);
        sh.positions.push_back(v[3 * k.v + 1]);
        sh.positions.push_back(v[3 * k.v + 2]);
        uint32_t id = static_cast<uint32_t>(sh.positions.size() / 3 - 1);
        seen.emplace(key, id);
        *out = id;
        return true;
    };
    for (size_t f = 0; f + 1 < fstart.size(); ++f) {
        const VIdx* w = fv.data() + fstart[f];
        const size_t cnt = fstart[f + 1] - fstart[f];
        for (size_t k = 2; k < cnt; ++k) {
            uint32_t a, b, c;
            if (!vertex(w[0], &a) || !vertex(w[k - 1], &b) || !vertex(w[k], &c)) return false;
            sh.indices.push_back(a);
            sh.indices.push_back(b);
            sh.indices.push_back(c);
            sh.material_ids.push_back(material);
        }
    }
    sh.name = name;
    shapes.push_back(std::move(sh));
    return true;
}

// pow(10, -k) and pow(5, e) exactly as tryParseDouble computes them (the same libm calls),
// tabulated once.
struct PowTables {
    double neg10[401];
    double pow5[801];   // e in [-400, 400]
    PowTables()
    {
        for (int k = 0; k <= 400; ++k) neg10[k] = pow(10.0, -k);
        for (int e = -400; e <= 400; ++e) pow5[e + 400] = pow(5.0, e);
    }
};
const PowTables& pow_tables()
{
    static const PowTables t;
    return t;
}

}  // namespace

bool parse_real(const char* s, const char* end, double* out)
{
    if (s >= end) return false;
    const char* p = s;
    bool negative = false;
    if (*p == '+' || *p == '-') {
        negative = (*p == '-');
        ++p;
    } else if (!digit(*p)) {
        return false;
    }
    double m = 0.0;
    int count = 0;
    bool inside = false;
    while ((inside = (p != end)) && digit(*p)) {
        m *= 10;
        m += static_cast<int>(*p - '0');
        ++p;
        ++count;
    }
    if (count == 0) return false;
    int e = 0;
    if (inside) {
        bool want_exponent = false;
        if (*p == '.') {
            ++p;
            int k = 1;
            while ((inside = (p != end)) && digit(*p)) {
                m += static_cast<int>(*p - '0') * (k <= 400 ? pow_tables().neg10[k] : pow(10.0, -k));
                ++k;
                ++p;
            }
            want_exponent = inside;
        } else if (*p == 'e' || *p == 'E') {
            want_exponent = true;
        }
        if (want_exponent && (*p == 'e' || *p == 'E')) {
            ++p;
            char esign = '+';
            if ((inside = (p != end)) && (*p == '+' || *p == '-')) {
                esign = *p;
                ++p;
            } else if (!digit(*p)) {
                return false;
            }
            int ne = 0;
            while ((inside = (p != end)) && digit(*p)) {
                e *= 10;
                e += static_cast<int>(*p - '0');
                ++p;
                ++ne;
            }
            e *= (esign == '+') ? 1 : -1;
            if (ne == 0) return false;
        }
    }
    *out = (negative ? -1 : 1) * ldexp(m * ((e >= -400 && e <= 400) ? pow_tables().pow5[e + 400] : pow(5.0, e)), e);
    return true;
}

ObjResult read_obj(const std::string& path, const std::string& mtl_basepath)
{
    ObjResult res;
    std::string text;
    if (!slurp(path, &text)) {
        res.message = "Cannot open file [" + path + "]\n";
        res.fatal = true;
        return res;
    }
    std::vector<float> v;
    int nvn = 0, nvt = 0;
    std::vector<VIdx> fv;
    std::vector<uint32_t> fstart(1, 0u);
    std::map<std::string, int> by_name;
    int material = -1;
    std::string name;
    std::string err;
    auto flush = [&]() -> bool {
        if (!emit_shape(fv, fstart, v, material, name, res.shapes, &err)) return false;
        fv.clear();
        fstart.assign(1, 0u);
        return true;
    };
    bool stop = false;
    for_each_line(text, [&](char* line) {
        if (stop) return;
        const char* t = line_start(line);
        if (!t) return;
        if (t[0] == 'v' && blank(t[1])) {
            t += 2;
            float x = next_real(t);
            float y = next_real(t);
            float z = next_real(t);
            v.push_back(x); v.push_back(y); v.push_back(z);
            return;
        }
        if (t[0] == 'v' && t[1] == 'n' && blank(t[2])) { ++nvn; return; }
        if (t[0] == 'v' && t[1] == 't' && blank(t[2])) { ++nvt; return; }
        if (t[0] == 'f' && blank(t[1])) {
            t += 2;
            t += strspn(t, " \t");
            while (!line_end(*t)) {
                fv.push_back(next_vidx(t, static_cast<int>(v.size() / 3), nvn, nvt));
                t += strspn(t, " \t\r");
            }
            fstart.push_back(static_cast<uint32_t>(fv.size()));
            return;
        }
        if (strncmp(t, "usemtl", 6) == 0 && blank(t[6])) {
            std::string mname = first_word(t + 7);
            if (!flush()) { res.message = err; res.fatal = true; stop = true; return; }
            auto it = by_name.find(mname);
            material = (it != by_name.end()) ? it->second : -1;
            return;
        }
        if (strncmp(t, "mtllib", 6) == 0 && blank(t[6])) {
            std::string lib = mtl_basepath + first_word(t + 7);
            if (!read_mtl(lib, res.materials, by_name)) {
                res.message = "WARN: Material file [ " + lib + " ] not found. Created a default material.";
                stop = true;   // tinyobj returns here: nothing after the mtllib line is read
                fv.clear();
                fstart.assign(1, 0u);
            }
            return;
        }
        if (t[0] == 'g' && blank(t[1])) {
            if (!flush()) { res.message = err; res.fatal = true; stop = true; return; }
            std::vector<std::string> words;
            while (!line_end(*t)) {
                t += strspn(t, " \t");
                size_t len = strcspn(t, " \t\r");
                words.emplace_back(t, len);
                t += len;
                t += strspn(t, " \t\r");
            }
            name = (words.size() > 1) ? words[1] : std::string();
            return;
        }
        if (t[0] == 'o' && blank(t[1])) {
            if (!flush()) { res.message = err; res.fatal = true; stop = true; return; }
            name = first_word(t + 2);
            return;
        }
    });
    if (stop) return res;   // fatal error, or tinyobj's early return at a missing mtllib
    if (!flush()) { res.message = err; res.fatal = true; }
    return res;
}

}  // namespace pt
