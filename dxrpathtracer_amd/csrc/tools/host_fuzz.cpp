// host_fuzz — sanitizer harness for the host-side parsers of libdxrpt_host (CPU only, no GPU).
//
// Built by scripts/asan_host.sh with -fsanitize=address,undefined together with the host sources.  For
// every input file (PNG / JPEG / DDS through dxrpt_host_texture_load, binary FBX through
// dxrpt_host_scene_load) it loads the file as is, then `--mutants` corrupted copies: truncations at
// seeded offsets and seeded byte flips (header-heavy: half the flips land in the first 4 KB).  Each load
// must either succeed or fail with a status and a message; a crash, hang or sanitizer report fails the
// run.  Prints one line per input: loads that succeeded / failed cleanly (an original the loaders do not
// support shows as REJECTED).
//
//   host_fuzz [--mutants N] [--seed S] [--tmp DIR] FILE...
#include <algorithm>
#include <cctype>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <functional>
#include <string>
#include <vector>

#include "../../../include/dxrpt.h"
#include "../../../include/dxrpt_host.h"

namespace {

uint64_t splitmix(uint64_t& s) {
    uint64_t z = (s += 0x9E3779B97F4A7C15ull);
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

bool read_file(const std::string& p, std::vector<uint8_t>& out) {
    FILE* f = std::fopen(p.c_str(), "rb");
    if (!f) return false;
    std::fseek(f, 0, SEEK_END);
    const long n = std::ftell(f);
    std::fseek(f, 0, SEEK_SET);
    out.resize(size_t(n > 0 ? n : 0));
    const bool ok = out.empty() || std::fread(out.data(), 1, out.size(), f) == out.size();
    std::fclose(f);
    return ok;
}

void write_file(const std::string& p, const uint8_t* d, size_t n) {
    FILE* f = std::fopen(p.c_str(), "wb");
    if (!f) {
        std::fprintf(stderr, "cannot write %s\n", p.c_str());
        std::exit(2);
    }
    if (n) std::fwrite(d, 1, n, f);
    std::fclose(f);
}

bool ends_with(const std::string& s, const char* suf) {
    const size_t n = std::strlen(suf);
    if (s.size() < n) return false;
    for (size_t i = 0; i < n; ++i)
        if (std::tolower(s[s.size() - n + i]) != suf[i]) return false;
    return true;
}

// One load of `path`; true = success.  Touches every output byte so the sanitizers see the buffers.
bool load(const std::string& path, bool fbx) {
    if (fbx) {
        dxrpt_host_model_settings st{};
        st.file_path = path.c_str();
        st.texture_dir = nullptr;
        st.scene_scale = 1.0f;
        st.force_srgb = 1;
        st.merge_meshes = 0;
        dxrpt_host_scene* sc = nullptr;
        if (dxrpt_host_scene_load(DXRPT_SCENE_WHITEFURNACE, &st, &sc) != DXRPT_OK) {
            if (!dxrpt_host_last_error()) std::abort();  // a failure must say why
            return false;
        }
        volatile float acc = 0.0f;
        for (uint32_t v = 0; v < sc->num_vertices; ++v) acc = acc + sc->vertices[v].Position[0];
        dxrpt_host_scene_destroy(sc);
        return true;
    }
    dxrpt_host_texture tex{};
    if (dxrpt_host_texture_load(path.c_str(), 1, &tex) != DXRPT_OK) {
        if (!dxrpt_host_last_error()) std::abort();
        return false;
    }
    const size_t bytes = size_t(tex.width) * tex.height * (tex.fmt == DXRPT_TEX_R8_UNORM ? 1u : 4u);
    volatile uint32_t acc = 0;
    const uint8_t* t = static_cast<const uint8_t*>(tex.texels);
    for (size_t i = 0; i < bytes; i += 61) acc = acc + t[i];
    if (bytes) acc = acc + t[bytes - 1];
    dxrpt_host_texture_free(&tex);
    return true;
}

}  // namespace

int main(int argc, char** argv) {
    int mutants = 64;
    uint64_t seed = 0x5EEDull;
    std::string tmp = "/tmp";
    std::vector<std::string> files;
    for (int i = 1; i < argc; ++i) {
        const std::string a = argv[i];
        if (a == "--mutants" && i + 1 < argc) mutants = std::atoi(argv[++i]);
        else if (a == "--seed" && i + 1 < argc) seed = std::strtoull(argv[++i], nullptr, 0);
        else if (a == "--tmp" && i + 1 < argc) tmp = argv[++i];
        else files.push_back(a);
    }
    int bad = 0;
    for (const std::string& path : files) {
        std::vector<uint8_t> data;
        if (!read_file(path, data)) {
            std::fprintf(stderr, "cannot read %s\n", path.c_str());
            ++bad;
            continue;
        }
        const bool fbx = ends_with(path, ".fbx");
        const std::string ext = path.substr(path.rfind('.'));
        const bool orig_ok = load(path, fbx);
        int ok = 0, failed = 0;
        uint64_t s = seed ^ std::hash<std::string>{}(path);
        for (int m = 0; m < mutants; ++m) {
            std::vector<uint8_t> mut = data;
            if (m % 3 == 0 && !mut.empty()) {  // truncation
                mut.resize(size_t(splitmix(s) % mut.size()));
            } else {                             // byte flips, half of them in the header region
                const int flips = 1 + int(splitmix(s) % 8);
                for (int k = 0; k < flips && !mut.empty(); ++k) {
                    const size_t lim = (k & 1) ? mut.size() : std::min<size_t>(mut.size(), 4096);
                    mut[splitmix(s) % lim] ^= uint8_t(1u + splitmix(s) % 255u);
                }
            }
            const std::string mp = tmp + "/host_fuzz_mutant" + ext;
            write_file(mp, mut.data(), mut.size());
            (load(mp, fbx) ? ok : failed)++;
        }
        std::printf("%-90s original %s, mutants: %d loaded, %d rejected\n", path.c_str(), orig_ok ? "loaded" : "REJECTED",
                    ok, failed);
        // an unsupported original (e.g. the reference's float DFG lookup table, not a material texture) is
        // reported, not a failure: the run fails only on unreadable inputs or a sanitizer report (abort)
    }
    return bad ? 1 : 0;
}
