// fbx.cpp — real-asset scene ingest: Model::CreateWithAssimp for binary FBX files.
//
// The reference loads its scenes through Assimp 4.1.0 (a prebuilt library, source not vendored:
// Externals/Assimp-4.1.0) in Model::CreateWithAssimp (Graphics/Model.cpp:435-606) with
//   ReadFile(path, 0) + ApplyPostProcessing(CalcTangentSpace | Triangulate | JoinIdenticalVertices |
//     MakeLeftHanded | RemoveRedundantMaterials | FlipUVs | FlipWindingOrder)        (:509-518)
//   MergeMeshes = false in DXRPathTracer (DXRPathTracer.cpp:951): no PreTransformVertices, so mesh
//     vertices stay in their geometry's local space (node transforms are not applied);
//   Mesh::InitFromAssimpMesh (:150-233): Position * SceneScale, bitangent * -1, UV set 0;
//   16-bit indices unless some mesh has more than 0xFFFF indices (:561-573);
//   LoadMaterialResources (:104-149): texture = TextureDir + file name, missing or unnamed ->
//     DefaultTextures (:74-82), albedo sRGB when ForceSRGB, textures shared by path.
// Restated here from Assimp's published behaviour for what those steps do to an FBX scene (parity
// with Assimp is unpinned: its exact float rounding, SpatialSort epsilons and visit orders are
// approximated):
//   * FBX binary 7.x reader (node records, typed properties, zlib-compressed arrays);
//   * FBX converter: one output vertex per polygon vertex (positions from Vertices through
//     PolygonVertexIndex, normals / tangents / binormals / UV set 0 per their Mapping/Reference
//     types), one mesh per (model, geometry, material index) with materials in first-use order and a
//     default material for geometry without one;
//   * post-processing in Assimp's step order: MakeLeftHanded (z of positions, normals, tangents,
//     bitangents negated), FlipUVs (v = 1 - v), FlipWindingOrder (face indices reversed),
//     Triangulate (quads split at their concave corner, larger polygons fanned), CalcTangentSpace
//     (only for meshes without tangents: per-face UV-derivative tangents projected per vertex, then
//     smoothed over vertices at the same position with normals within 0.9999 and tangents within
//     45 degrees), JoinIdenticalVertices (first-occurrence order, 1e-5 tolerance).
// Texture slots follow Assimp's FBX material mapping: DiffuseColor -> albedo, NormalMap or Bump ->
// normal, ShininessExponent -> roughness, AmbientColor -> metallic, TransparentColor -> opacity,
// EmissiveColor -> emissive (Model.cpp:533-549).  Texture files: DDS (dds.cpp); other formats the
// reference decodes through WIC are not supported here and fail the load.
#include <zlib.h>

#include <algorithm>
#include <array>
#include <cmath>
#include <cstring>
#include <fstream>
#include <map>
#include <memory>
#include <string>
#include <unordered_map>
#include <vector>

#include "scene_builder.h"

namespace dxrpt_host {

namespace fbx {

struct Error : std::runtime_error {
    using std::runtime_error::runtime_error;
};

// ---- binary FBX document ---------------------------------------------------------------------------
struct Prop {
    char type = 0;
    int64_t i = 0;
    double d = 0.0;
    std::string s;               // S / R
    std::vector<double> darr;    // f / d arrays
    std::vector<int64_t> iarr;   // i / l / b arrays
};

struct Node {
    std::string name;
    std::vector<Prop> props;
    std::vector<Node> children;

    const Node* child(const char* n) const {
        for (const Node& c : children)
            if (c.name == n) return &c;
        return nullptr;
    }
    std::vector<const Node*> all(const char* n) const {
        std::vector<const Node*> out;
        for (const Node& c : children)
            if (c.name == n) out.push_back(&c);
        return out;
    }
};

class Reader {
  public:
    explicit Reader(std::vector<uint8_t> bytes) : d_(std::move(bytes)) {}

    Node parse() {
        static const char kMagic[] = "Kaydara FBX Binary  ";
        if (d_.size() < 27 || std::memcmp(d_.data(), kMagic, 20) != 0) throw Error("not a binary FBX file");
        version_ = u32(23);
        Node root;
        size_t off = 27;
        while (true) {
            Node n;
            if (!record(off, n)) break;
            root.children.push_back(std::move(n));
        }
        return root;
    }
    uint32_t version() const { return version_; }

  private:
    std::vector<uint8_t> d_;
    uint32_t version_ = 0;

    void need(size_t off, size_t n) const {
        if (off + n > d_.size()) throw Error("truncated FBX file");
    }
    uint32_t u32(size_t o) const {
        need(o, 4);
        uint32_t v;
        std::memcpy(&v, d_.data() + o, 4);
        return v;
    }
    uint64_t u64(size_t o) const {
        need(o, 8);
        uint64_t v;
        std::memcpy(&v, d_.data() + o, 8);
        return v;
    }

    // Reads one node record at `off` (advances it).  Returns false on the null record.
    bool record(size_t& off, Node& n) {
        const bool wide = version_ >= 7500;
        const uint64_t end = wide ? u64(off) : u32(off);
        const uint64_t nprops = wide ? u64(off + 8) : u32(off + 4);
        off += wide ? 24 : 12;
        need(off, 1);
        const uint8_t nl = d_[off++];
        if (end == 0) return false;
        need(off, nl);
        n.name.assign(reinterpret_cast<const char*>(d_.data() + off), nl);
        off += nl;
        for (uint64_t k = 0; k < nprops; ++k) n.props.push_back(prop(off));
        while (off < end) {
            Node c;
            if (!record(off, c)) break;
            n.children.push_back(std::move(c));
        }
        off = size_t(end);
        return true;
    }

    Prop prop(size_t& off) {
        need(off, 1);
        Prop p;
        p.type = char(d_[off++]);
        auto scalar = [&](size_t sz) {
            need(off, sz);
            const uint8_t* q = d_.data() + off;
            off += sz;
            return q;
        };
        switch (p.type) {
            case 'Y': { int16_t v; std::memcpy(&v, scalar(2), 2); p.i = v; break; }
            case 'C': p.i = *scalar(1); break;
            case 'I': { int32_t v; std::memcpy(&v, scalar(4), 4); p.i = v; break; }
            case 'L': { int64_t v; std::memcpy(&v, scalar(8), 8); p.i = v; break; }
            case 'F': { float v; std::memcpy(&v, scalar(4), 4); p.d = v; break; }
            case 'D': { double v; std::memcpy(&v, scalar(8), 8); p.d = v; break; }
            case 'S':
            case 'R': {
                const uint32_t len = u32(off);
                off += 4;
                need(off, len);
                p.s.assign(reinterpret_cast<const char*>(d_.data() + off), len);
                off += len;
                break;
            }
            case 'f': case 'd': case 'i': case 'l': case 'b': {
                const uint32_t count = u32(off), enc = u32(off + 4), clen = u32(off + 8);
                off += 12;
                need(off, clen);
                const size_t esz = (p.type == 'd' || p.type == 'l') ? 8 : (p.type == 'b' ? 1 : 4);
                std::vector<uint8_t> raw(size_t(count) * esz);
                if (enc == 0) {
                    if (clen < raw.size()) throw Error("FBX array shorter than its count");
                    std::memcpy(raw.data(), d_.data() + off, raw.size());
                } else if (enc == 1) {
                    uLongf dlen = uLongf(raw.size());
                    if (uncompress(raw.data(), &dlen, d_.data() + off, uLong(clen)) != Z_OK || dlen != raw.size())
                        throw Error("FBX array: zlib inflate failed");
                } else {
                    throw Error("FBX array: unknown encoding");
                }
                off += clen;
                for (uint32_t k = 0; k < count; ++k) {
                    const uint8_t* q = raw.data() + size_t(k) * esz;
                    if (p.type == 'f') { float v; std::memcpy(&v, q, 4); p.darr.push_back(v); }
                    else if (p.type == 'd') { double v; std::memcpy(&v, q, 8); p.darr.push_back(v); }
                    else if (p.type == 'i') { int32_t v; std::memcpy(&v, q, 4); p.iarr.push_back(v); }
                    else if (p.type == 'l') { int64_t v; std::memcpy(&v, q, 8); p.iarr.push_back(v); }
                    else p.iarr.push_back(*q);
                }
                break;
            }
            default: throw Error(std::string("FBX: unknown property type '") + p.type + "'");
        }
        return p;
    }
};

const std::vector<double>& darr(const Node* n) {
    static const std::vector<double> empty;
    return (n && !n->props.empty()) ? n->props[0].darr : empty;
}
const std::vector<int64_t>& iarr(const Node* n) {
    static const std::vector<int64_t> empty;
    return (n && !n->props.empty()) ? n->props[0].iarr : empty;
}
std::string str(const Node* n) { return (n && !n->props.empty()) ? n->props[0].s : std::string(); }

// ---- mesh conversion -------------------------------------------------------------------------------
struct Vtx {
    V3 p, n, t, b;
    float u = 0, v = 0;
};

// A per-polygon-vertex attribute layer (LayerElementNormal / Tangent / Binormal / UV).
template <int N>
bool read_layer(const Node* le, const char* data_name, const char* index_name, const std::vector<int64_t>& pvi_vertex,
                const std::vector<uint32_t>& poly_of, std::vector<std::array<float, N>>& out) {
    if (!le) return false;
    const std::string mapping = str(le->child("MappingInformationType"));
    const std::string reference = str(le->child("ReferenceInformationType"));
    const std::vector<double>& data = darr(le->child(data_name));
    const std::vector<int64_t>& index = iarr(index_name ? le->child(index_name) : nullptr);
    const size_t n = pvi_vertex.size();
    out.assign(n, std::array<float, N>{});
    for (size_t k = 0; k < n; ++k) {
        size_t e;
        if (mapping == "ByPolygonVertex") e = k;
        else if (mapping == "ByVertex" || mapping == "ByVertice") e = size_t(pvi_vertex[k]);
        else if (mapping == "ByPolygon") e = poly_of[k];
        else if (mapping == "AllSame") e = 0;
        else throw Error("FBX: unsupported mapping type " + mapping);
        if (reference == "IndexToDirect" || reference == "Index") {
            if (e >= index.size()) throw Error(std::string("FBX: ") + index_name + " out of range");
            e = size_t(index[e]);
        }
        if ((e + 1) * N > data.size()) throw Error(std::string("FBX: ") + data_name + " out of range");
        for (int j = 0; j < N; ++j) out[k][j] = float(data[e * N + j]);
    }
    return true;
}

const Node* layer_element(const Node& geo, const char* type, int typed_index) {
    for (const Node* le : geo.all(type))
        if (!le->props.empty() && le->props[0].i == typed_index) return le;
    return nullptr;
}

struct MeshOut {
    std::vector<Vtx> verts;
    std::vector<std::vector<uint32_t>> faces;
    uint32_t material = 0;  // index into the scene's material list
    bool has_tangents = false;
    bool has_uv = false;
};

float len(V3 a) { return std::sqrt(dot(a, a)); }
V3 norm(V3 a) {  // aiVector3D::Normalize: v / |v| (NaN / inf for zero vectors, as in Assimp)
    const float l = len(a);
    return a * (1.0f / l);
}
bool special(V3 a) { return !std::isfinite(a.x) || !std::isfinite(a.y) || !std::isfinite(a.z); }

// TriangulateProcess: quads split at the concave corner (if any), larger polygons fanned.
void triangulate(MeshOut& m) {
    std::vector<std::vector<uint32_t>> out;
    for (const auto& f : m.faces) {
        if (f.size() < 3) continue;
        if (f.size() == 3) {
            out.push_back(f);
            continue;
        }
        if (f.size() == 4) {
            unsigned start = 0;
            for (unsigned i = 0; i < 4; ++i) {
                const V3 v = m.verts[f[i]].p;
                const V3 l = norm(m.verts[f[(i + 3) % 4]].p - v), dg = norm(m.verts[f[(i + 2) % 4]].p - v),
                         r = norm(m.verts[f[(i + 1) % 4]].p - v);
                const float angle = std::acos(dot(l, dg)) + std::acos(dot(r, dg));
                if (angle > 3.14159265358979f) {
                    start = i;
                    break;
                }
            }
            out.push_back({f[start], f[(start + 1) % 4], f[(start + 2) % 4]});
            out.push_back({f[start], f[(start + 2) % 4], f[(start + 3) % 4]});
            continue;
        }
        for (size_t i = 1; i + 1 < f.size(); ++i) out.push_back({f[0], f[i], f[i + 1]});
    }
    m.faces.swap(out);
}

// Vertices within `eps` of a position, in the order of their projection on a fixed plane normal
// (Assimp's SpatialSort).
struct SpatialSort {
    V3 pn{0.8523f, 0.34321f, 0.5736f};
    std::vector<std::pair<float, uint32_t>> keys;
    const std::vector<Vtx>* v = nullptr;
    void build(const std::vector<Vtx>& verts) {
        v = &verts;
        keys.clear();
        for (uint32_t i = 0; i < verts.size(); ++i) keys.push_back({dot(verts[i].p, pn), i});
        std::stable_sort(keys.begin(), keys.end(), [](const auto& a, const auto& b) { return a.first < b.first; });
    }
    void find(V3 p, float eps, std::vector<uint32_t>& out) const {
        out.clear();
        const float d = dot(p, pn);
        auto it = std::lower_bound(keys.begin(), keys.end(), d - eps, [](const auto& a, float x) { return a.first < x; });
        for (; it != keys.end() && it->first < d + eps; ++it) {
            const V3 q = (*v)[it->second].p - p;
            if (dot(q, q) < eps * eps) out.push_back(it->second);
        }
    }
};

float position_epsilon(const std::vector<Vtx>& verts) {
    V3 lo{1e30f, 1e30f, 1e30f}, hi{-1e30f, -1e30f, -1e30f};
    for (const Vtx& x : verts) {
        lo = {std::min(lo.x, x.p.x), std::min(lo.y, x.p.y), std::min(lo.z, x.p.z)};
        hi = {std::max(hi.x, x.p.x), std::max(hi.y, x.p.y), std::max(hi.z, x.p.z)};
    }
    return len(hi - lo) * 1e-4f;
}

// CalcTangentsProcess (meshes without tangents).
void calc_tangents(MeshOut& m) {
    if (m.has_tangents || !m.has_uv) return;  // Assimp needs UV channel 0 to compute tangents
    std::vector<Vtx>& V = m.verts;
    for (const auto& f : m.faces) {
        const uint32_t p0 = f[0], p1 = f[1], p2 = f[2];
        const V3 v = V[p1].p - V[p0].p, w = V[p2].p - V[p0].p;
        float sx = V[p1].u - V[p0].u, sy = V[p1].v - V[p0].v;
        float tx = V[p2].u - V[p0].u, ty = V[p2].v - V[p0].v;
        const float dirCorrection = (tx * sy - ty * sx) < 0.0f ? -1.0f : 1.0f;
        if (sx * ty == sy * tx) {
            sx = 0.0f; sy = 1.0f; tx = 1.0f; ty = 0.0f;
        }
        const V3 tangent{(w.x * sy - v.x * ty) * dirCorrection, (w.y * sy - v.y * ty) * dirCorrection,
                         (w.z * sy - v.z * ty) * dirCorrection};
        const V3 bitangent{(w.x * sx - v.x * tx) * dirCorrection, (w.y * sx - v.y * tx) * dirCorrection,
                           (w.z * sx - v.z * tx) * dirCorrection};
        for (uint32_t p : f) {
            const V3 n = V[p].n;
            V3 lt = norm(tangent - n * dot(tangent, n));
            V3 lb = norm(bitangent - n * dot(bitangent, n));
            const bool it = special(lt), ib = special(lb);
            if (it != ib) {
                if (it) lt = norm(cross(n, lb));
                else lb = norm(cross(lt, n));
            }
            V[p].t = lt;
            V[p].b = lb;
        }
    }
    SpatialSort ss;
    ss.build(V);
    const float eps = position_epsilon(V);
    const float fLimit = std::cos(45.0f * 3.14159265358979f / 180.0f), angleEpsilon = 0.9999f;
    std::vector<bool> done(V.size(), false);
    std::vector<uint32_t> found, close;
    for (uint32_t a = 0; a < V.size(); ++a) {
        if (done[a]) continue;
        const Vtx o = V[a];
        ss.find(o.p, eps, found);
        close.assign(1, a);
        for (uint32_t idx : found) {
            if (done[idx]) continue;
            if (dot(V[idx].n, o.n) < angleEpsilon) continue;
            if (dot(V[idx].t, o.t) < fLimit) continue;
            if (dot(V[idx].b, o.b) < fLimit) continue;
            close.push_back(idx);
            done[idx] = true;
        }
        V3 st{0, 0, 0}, sb{0, 0, 0};
        for (uint32_t c : close) {
            st = st + V[c].t;
            sb = sb + V[c].b;
        }
        st = norm(st);
        sb = norm(sb);
        for (uint32_t c : close) {
            V[c].t = st;
            V[c].b = sb;
        }
    }
    m.has_tangents = true;
}

// JoinVerticesProcess: identical vertices (position within the SpatialSort epsilon, every other
// attribute within 1e-5) merge into the first occurrence.
void join_vertices(MeshOut& m) {
    const std::vector<Vtx>& V = m.verts;
    SpatialSort ss;
    ss.build(V);
    const float eps = position_epsilon(V);
    const float sq = 1e-5f * 1e-5f;
    auto close3 = [&](V3 a, V3 b) {
        const V3 d = a - b;
        return dot(d, d) <= sq;
    };
    std::vector<Vtx> uniq;
    std::vector<uint32_t> replace(V.size(), ~0u);
    std::vector<uint32_t> found;
    for (uint32_t a = 0; a < V.size(); ++a) {
        ss.find(V[a].p, eps, found);
        uint32_t hit = ~0u;
        for (uint32_t c : found) {
            if (c >= a || replace[c] == ~0u) continue;
            const Vtx& u = uniq[replace[c]];
            const float du = u.u - V[a].u, dv = u.v - V[a].v;
            if (close3(u.n, V[a].n) && du * du + dv * dv <= sq && close3(u.t, V[a].t) && close3(u.b, V[a].b)) {
                hit = replace[c];
                break;
            }
        }
        if (hit == ~0u) {
            hit = uint32_t(uniq.size());
            uniq.push_back(V[a]);
        }
        replace[a] = hit;
    }
    for (auto& f : m.faces)
        for (auto& i : f) i = replace[i];
    m.verts.swap(uniq);
}

}  // namespace fbx

// Builds the scene into B.  Returns the maximum index count of a mesh (index-size choice).
size_t load_fbx_scene(const std::string& path, const std::string& texture_dir, float scene_scale, bool force_srgb,
                      SceneBuilder& B) {
    using namespace fbx;
    std::ifstream f(path, std::ios::binary);
    if (!f) throw Error("Model file with path '" + path + "' does not exist");
    Reader rd(std::vector<uint8_t>((std::istreambuf_iterator<char>(f)), std::istreambuf_iterator<char>()));
    const Node doc = rd.parse();
    const Node* objects = doc.child("Objects");
    const Node* connections = doc.child("Connections");
    if (!objects) throw Error("FBX: no Objects section");

    std::unordered_map<int64_t, const Node*> byid;
    for (const Node& o : objects->children)
        if (!o.props.empty()) byid[o.props[0].i] = &o;
    struct Conn {
        std::string kind;
        int64_t child, parent;
        std::string prop;
    };
    std::vector<Conn> conns;
    if (connections)
        for (const Node* c : connections->all("C"))
            if (c->props.size() >= 3)
                conns.push_back({c->props[0].s, c->props[1].i, c->props[2].i, c->props.size() > 3 ? c->props[3].s : ""});
    auto children_of = [&](int64_t parent, const char* cls) {
        std::vector<const Node*> out;
        for (const Conn& c : conns)
            if (c.kind == "OO" && c.parent == parent) {
                auto it = byid.find(c.child);
                if (it != byid.end() && it->second->name == cls) out.push_back(it->second);
            }
        return out;
    };

    // ---- models in hierarchy order (root id 0, children in connection order), their geometry
    std::vector<const Node*> models;
    std::vector<int64_t> stack{0};
    std::vector<int64_t> order;
    while (!stack.empty()) {  // depth-first, children in connection order
        const int64_t id = stack.back();
        stack.pop_back();
        if (id != 0) order.push_back(id);
        std::vector<int64_t> kids;
        for (const Conn& c : conns)
            if (c.kind == "OO" && c.parent == id) {
                auto it = byid.find(c.child);
                if (it != byid.end() && it->second->name == "Model") kids.push_back(c.child);
            }
        for (auto it = kids.rbegin(); it != kids.rend(); ++it) stack.push_back(*it);
    }
    for (int64_t id : order) models.push_back(byid[id]);

    // ---- materials (first use order) and their texture file names per slot
    enum Slot { Albedo, Normal, Roughness, Metallic, Opacity, Emissive, NumSlots };
    struct Mat {
        std::string tex[NumSlots];
    };
    std::vector<Mat> mats;
    std::map<int64_t, uint32_t> mat_index;
    int default_mat = -1;
    auto texture_name = [&](int64_t material_id, const char* prop) -> std::string {
        for (const Conn& c : conns)
            if (c.kind == "OP" && c.parent == material_id && c.prop == prop) {
                auto it = byid.find(c.child);
                if (it == byid.end() || it->second->name != "Texture") continue;
                std::string name = str(it->second->child("RelativeFilename"));
                if (name.empty()) name = str(it->second->child("FileName"));
                const size_t s = name.find_last_of("/\\");  // GetFileName
                return s == std::string::npos ? name : name.substr(s + 1);
            }
        return std::string();
    };
    auto material_for = [&](const Node* m) -> uint32_t {
        if (!m) {
            if (default_mat < 0) {
                default_mat = int(mats.size());
                mats.push_back(Mat{});
            }
            return uint32_t(default_mat);
        }
        const int64_t id = m->props[0].i;
        auto it = mat_index.find(id);
        if (it != mat_index.end()) return it->second;
        Mat mt;
        mt.tex[Albedo] = texture_name(id, "DiffuseColor");
        mt.tex[Normal] = texture_name(id, "NormalMap");
        if (mt.tex[Normal].empty()) mt.tex[Normal] = texture_name(id, "Bump");
        mt.tex[Roughness] = texture_name(id, "ShininessExponent");
        mt.tex[Metallic] = texture_name(id, "AmbientColor");
        mt.tex[Opacity] = texture_name(id, "TransparentColor");
        mt.tex[Emissive] = texture_name(id, "EmissiveColor");
        const uint32_t k = uint32_t(mats.size());
        mats.push_back(mt);
        mat_index[id] = k;
        return k;
    };

    std::vector<MeshOut> meshes;
    for (const Node* model : models) {
        const std::vector<const Node*> model_mats = children_of(model->props[0].i, "Material");
        for (const Node* geo : children_of(model->props[0].i, "Geometry")) {
            if (geo->props.size() < 3 || geo->props[2].s != "Mesh") continue;
            const std::vector<double>& P = darr(geo->child("Vertices"));
            const std::vector<int64_t>& PVI = iarr(geo->child("PolygonVertexIndex"));
            if (P.empty() || PVI.empty()) continue;
            std::vector<int64_t> pv(PVI.size());
            std::vector<uint32_t> poly_of(PVI.size());
            std::vector<std::pair<uint32_t, uint32_t>> polys;  // (first polygon vertex, count)
            uint32_t start = 0, pi = 0;
            for (size_t k = 0; k < PVI.size(); ++k) {
                const int64_t v = PVI[k];
                pv[k] = v < 0 ? ~v : v;
                if (size_t(pv[k]) * 3 + 2 >= P.size()) throw Error("FBX: polygon vertex index out of range");
                poly_of[k] = pi;
                if (v < 0) {
                    polys.push_back({start, uint32_t(k + 1 - start)});
                    start = uint32_t(k + 1);
                    ++pi;
                }
            }
            std::vector<std::array<float, 3>> N, T, Bn;
            std::vector<std::array<float, 2>> UV;
            const bool hasN = read_layer<3>(layer_element(*geo, "LayerElementNormal", 0), "Normals", "NormalsIndex", pv, poly_of, N);
            const bool hasT = read_layer<3>(layer_element(*geo, "LayerElementTangent", 0), "Tangents", "TangentsIndex", pv, poly_of, T);
            const bool hasB = read_layer<3>(layer_element(*geo, "LayerElementBinormal", 0), "Binormals", "BinormalsIndex", pv, poly_of, Bn);
            const bool hasUV = read_layer<2>(layer_element(*geo, "LayerElementUV", 0), "UV", "UVIndex", pv, poly_of, UV);
            // material per polygon
            std::vector<int64_t> poly_mat(polys.size(), 0);
            if (const Node* lm = layer_element(*geo, "LayerElementMaterial", 0)) {
                const std::string mapping = str(lm->child("MappingInformationType"));
                const std::vector<int64_t>& mi = iarr(lm->child("Materials"));
                for (size_t q = 0; q < polys.size(); ++q)
                    poly_mat[q] = mi.empty() ? 0 : (mapping == "AllSame" ? mi[0] : mi[std::min(q, mi.size() - 1)]);
            }
            std::vector<int64_t> used(poly_mat.begin(), poly_mat.end());
            std::sort(used.begin(), used.end());
            used.erase(std::unique(used.begin(), used.end()), used.end());
            for (int64_t mi : used) {
                MeshOut m;
                m.material = material_for(mi >= 0 && size_t(mi) < model_mats.size() ? model_mats[size_t(mi)] : nullptr);
                m.has_tangents = hasT && hasB;
                m.has_uv = hasUV;
                for (size_t q = 0; q < polys.size(); ++q) {
                    if (poly_mat[q] != mi) continue;
                    std::vector<uint32_t> face;
                    for (uint32_t k = polys[q].first; k < polys[q].first + polys[q].second; ++k) {
                        Vtx x;
                        x.p = V3{float(P[pv[k] * 3 + 0]), float(P[pv[k] * 3 + 1]), float(P[pv[k] * 3 + 2])};
                        if (hasN) x.n = V3{N[k][0], N[k][1], N[k][2]};
                        if (m.has_tangents) {
                            x.t = V3{T[k][0], T[k][1], T[k][2]};
                            x.b = V3{Bn[k][0], Bn[k][1], Bn[k][2]};
                        }
                        if (hasUV) {
                            x.u = UV[k][0];
                            x.v = UV[k][1];
                        }
                        face.push_back(uint32_t(m.verts.size()));
                        m.verts.push_back(x);
                    }
                    m.faces.push_back(std::move(face));
                }
                meshes.push_back(std::move(m));
            }
        }
    }
    if (meshes.empty()) throw Error("Scene " + path + " has no meshes");

    // ---- post-processing (Assimp step order)
    size_t max_indices = 0;
    for (MeshOut& m : meshes) {
        for (Vtx& x : m.verts) {  // MakeLeftHanded, FlipUVs
            x.p.z = -x.p.z;
            x.n.z = -x.n.z;
            x.t.z = -x.t.z;
            x.b.z = -x.b.z;
            x.v = 1.0f - x.v;
        }
        for (auto& face : m.faces) std::reverse(face.begin(), face.end());  // FlipWindingOrder
        triangulate(m);
        calc_tangents(m);
        join_vertices(m);
        max_indices = std::max(max_indices, m.faces.size() * 3);
    }

    // ---- LoadMaterialResources: textures by path, defaults for missing names/files
    std::map<std::string, uint32_t> tex_by_path;
    const char* default_names[NumSlots] = {"DefaultBaseColor", "DefaultNormalMap", "DefaultRoughness", "DefaultBlack", "",
                                           "DefaultBlack"};
    auto default_tex = [&](int slot) -> uint32_t {
        const std::string key = std::string("<default>") + default_names[slot] + (slot == Albedo && force_srgb ? "_srgb" : "");
        auto it = tex_by_path.find(key);
        if (it != tex_by_path.end()) return it->second;
        Texture t;
        if (slot == Albedo) t = solid_rgba(0xC0, 0xC0, 0xC0, 0xFF, force_srgb ? DXRPT_TEX_RGBA8_SRGB : DXRPT_TEX_RGBA8_UNORM);
        else if (slot == Normal) t = solid_rgba(0x7F, 0x7F, 0xFF, 0xFF);
        else if (slot == Roughness) t = solid_rgba(0x40, 0x40, 0x40, 0xFF);
        else t = solid_rgba(0x00, 0x00, 0x00, 0xFF);
        const uint32_t k = B.add_texture(std::move(t));
        tex_by_path[key] = k;
        return k;
    };
    std::vector<uint32_t> mat_ids;
    for (const Mat& mt : mats) {
        uint32_t idx[NumSlots];
        for (int s = 0; s < NumSlots; ++s) {
            std::string file = mt.tex[s].empty() ? std::string() : texture_dir + mt.tex[s];
            bool exists = false;
            if (!file.empty()) {
                std::ifstream probe(file, std::ios::binary);
                exists = bool(probe);
            }
            if (!exists) {
                idx[s] = s == Opacity ? DXRPT_INVALID_INDEX : default_tex(s);
                continue;
            }
            const bool srgb = force_srgb && s == Albedo;
            const std::string key = file + (srgb ? "|srgb" : "");
            auto it = tex_by_path.find(key);
            if (it != tex_by_path.end()) {
                idx[s] = it->second;
                continue;
            }
            Texture t;
            std::string err;
            if (!load_image(file, srgb, t, err)) throw Error(err);  // DDS / PNG / JPEG (WIC in the reference)
            idx[s] = B.add_texture(std::move(t));
            tex_by_path[key] = idx[s];
        }
        mat_ids.push_back(B.add_material(idx[Albedo], idx[Normal], idx[Roughness], idx[Metallic], idx[Opacity], idx[Emissive]));
    }

    // ---- Mesh::InitFromAssimpMesh
    for (const MeshOut& m : meshes) {
        B.begin_mesh(mat_ids[m.material]);
        for (const Vtx& x : m.verts)
            B.vtx(x.p * scene_scale, x.n, x.u, x.v, x.t, x.b * -1.0f);
        for (const auto& face : m.faces) B.tri(face[0], face[1], face[2]);
        B.end_mesh();
    }
    return max_indices;
}

}  // namespace dxrpt_host
