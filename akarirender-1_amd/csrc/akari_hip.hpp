// akari_hip.hpp — C++17 host adapter over the C-ABI (include/akr_hip.h).
//
// Mirrors the reference's plug-in interface for the hot path so the MI355X backend drops in
// beside EmbreeAccelerator / BVHAccelerator and the CPU/GPU integrators:
//
//   akari::hip::HipAccelerator   ~ Accelerator concept: build(scene), intersect(ray, isct),
//                                  occlude(ray)   (kernel/bvh-accelerator.h:673-682,
//                                  kernel/embree.inl:37-45; dispatch kernel/scene.cpp:26-81)
//   akari::hip::HipPathTracer    ~ gpu::PathTracer / cpu::PathTracer with
//                                  render(scene, film)  (kernel/integrators/gpu/integrator.h:39-59,
//                                  core/nodes/integrator.cpp:50-84)
//   akari::hip::Film             ~ Film<C>: Pixel{radiance, weight} (core/film.h:31-113)
//
// Errors: a non-zero C-ABI status becomes std::runtime_error (the AKR_ASSERT_THROW convention,
// common/panic.h:52-57) carrying akr_hip_last_error().
#pragma once
#include <cstdint>
#include <cstdio>
#include <stdexcept>
#include <cmath>
#include <algorithm>
#include <string>
#include <limits>
#include <vector>

#include "../../include/akr_hip.h"

namespace akari::hip {

inline void check(akr_hip_ctx *ctx, int status, const char *what) {
    if (status != 0)
        throw std::runtime_error(std::string(what) + ": " + (ctx ? akr_hip_last_error(ctx) : "no context"));
}

// Flat mesh view, the MeshInstance<C> fields (kernel/instance.h:30-35).
struct MeshView {
    const float *vertices = nullptr;     // 3 * n_vertices
    uint64_t n_vertices = 0;
    const int32_t *indices = nullptr;    // 3 * n_triangles
    const float *normals = nullptr;      // 9 * n_triangles
    const float *texcoords = nullptr;    // 6 * n_triangles
    const int32_t *material_indices = nullptr;
    uint64_t n_triangles = 0;
    std::vector<int32_t> material_slots; // mesh-local material index -> scene material index
};

struct SceneDesc {
    std::vector<MeshView> meshes;
    std::vector<akr_texture> textures;
    std::vector<akr_material> materials;
    std::vector<akr_area_light> lights;
    std::vector<float> light_power;      // SceneNode::compile power weights (core/nodes/scene.cpp:72-87)
    akr_camera camera{};
};

class HipAccelerator {
  public:
    explicit HipAccelerator(int device = 0) {
        int st = akr_hip_create(device, &ctx_);
        if (st != 0) throw std::runtime_error("akr_hip_create failed (no HIP device " + std::to_string(device) + ")");
    }
    ~HipAccelerator() { akr_hip_destroy(ctx_); }
    HipAccelerator(const HipAccelerator &) = delete;
    HipAccelerator &operator=(const HipAccelerator &) = delete;

    // BVHAccelerator::build(Scene<C>&): uploads the flat scene and builds the BVH on the host.
    void build(const SceneDesc &s, const akr_build_params *params = nullptr) {
        check(ctx_, akr_hip_upload_textures(ctx_, s.textures.data(), (int32_t)s.textures.size()), "upload_textures");
        check(ctx_, akr_hip_upload_materials(ctx_, s.materials.data(), (int32_t)s.materials.size()), "upload_materials");
        for (const auto &m : s.meshes) {
            int32_t gid = -1;
            check(ctx_, akr_hip_upload_mesh(ctx_, m.vertices, m.n_vertices, m.indices, m.normals, m.texcoords,
                                            m.material_indices, m.n_triangles, m.material_slots.data(),
                                            (int32_t)m.material_slots.size(), &gid),
                  "upload_mesh");
        }
        check(ctx_, akr_hip_upload_lights(ctx_, s.lights.data(), (int32_t)s.lights.size(), s.light_power.data()),
              "upload_lights");
        check(ctx_, akr_hip_set_camera(ctx_, &s.camera), "set_camera");
        check(ctx_, akr_hip_build_accel(ctx_, params), "build_accel");
    }
    // Scene<C>::intersect(ray, isct) -> bool (kernel/scene.cpp:26-45), batched on the device.
    void intersect(const std::vector<akr_ray> &rays, std::vector<akr_hit> &hits) const {
        hits.resize(rays.size());
        check(ctx_, akr_hip_trace(ctx_, rays.data(), rays.size(), hits.data(), 0), "trace");
    }
    bool intersect(const akr_ray &ray, akr_hit *isct) const {
        check(ctx_, akr_hip_trace(ctx_, &ray, 1, isct, 0), "trace");
        return isct->geom_id != -1 && isct->prim_id != -1;   // Intersection::hit (scene.h:48)
    }
    // Scene<C>::occlude(ray) -> bool (kernel/scene.cpp:46-63)
    void occlude(const std::vector<akr_ray> &rays, std::vector<uint8_t> &occluded) const {
        std::vector<akr_hit> hits(rays.size());
        check(ctx_, akr_hip_trace(ctx_, rays.data(), rays.size(), hits.data(), 1), "trace(any)");
        occluded.resize(rays.size());
        for (size_t i = 0; i < rays.size(); i++) occluded[i] = hits[i].geom_id != -1;
    }
    bool occlude(const akr_ray &ray) const {
        akr_hit h;
        check(ctx_, akr_hip_trace(ctx_, &ray, 1, &h, 1), "trace(any)");
        return h.geom_id != -1;
    }
    akr_accel_info info() const {
        akr_accel_info i;
        check(ctx_, akr_hip_accel_info(ctx_, &i), "accel_info");
        return i;
    }
    akr_hip_ctx *handle() const { return ctx_; }

  private:
    akr_hip_ctx *ctx_ = nullptr;
};

// Film<C> (core/film.h:72-113): per-pixel sum of radiance and weight; value = radiance / weight.
struct Film {
    int width = 0, height = 0;
    std::vector<float> radiance, weight;
    Film(int w, int h) : width(w), height(h), radiance(3 * (size_t)w * h, 0.0f), weight((size_t)w * h, 0.0f) {}
    void pixel(int x, int y, float rgb[3]) const {
        size_t p = (size_t)x + (size_t)y * width;
        float w = weight[p];
        for (int c = 0; c < 3; c++) rgb[c] = w != 0 ? radiance[3 * p + c] / w : radiance[3 * p + c];
    }
    // Film::write_image (core/film.h:97-113) with GammaCorrection (common/color.h:58-61) and the
    // 8-bit quantisation of DefaultImageWriter (core/image.cpp:38-60): row-major RGB bytes.  pow
    // in f64 rounded to f32 (the correctly rounded powf); identical to akari_amd/film.py.
    std::vector<uint8_t> srgb8() const {
        std::vector<uint8_t> out(3 * (size_t)width * height);
        for (int y = 0; y < height; y++)
            for (int x = 0; x < width; x++) {
                float rgb[3];
                pixel(x, y, rgb);
                for (int c = 0; c < 3; c++) {
                    const float L = rgb[c];
                    const float p = (float)std::pow((double)L, (double)(1.0f / 2.4f));
                    float s = L < 0.0031308f ? L * 12.92f : 1.055f * p - 0.055f;
                    if (!(s >= 0.0f)) s = 0.0f;  // clamp to [0, 1] (NaN -> 0)
                    if (s > 1.0f) s = 1.0f;
                    const int q = (int)std::round((double)s * 255.5);
                    out[3 * ((size_t)x + (size_t)y * width) + c] = (uint8_t)std::min(255, std::max(0, q));
                }
            }
        return out;
    }
    // 8-bit RGB PNG with stored (uncompressed) deflate blocks: no codec dependency.
    bool write_png(const std::string &path) const {
        const std::vector<uint8_t> rgb = srgb8();
        std::vector<uint8_t> raw;
        raw.reserve((size_t)height * (1 + 3 * (size_t)width));
        for (int y = 0; y < height; y++) {
            raw.push_back(0);  // filter type 0
            raw.insert(raw.end(), rgb.begin() + 3 * (size_t)y * width, rgb.begin() + 3 * (size_t)(y + 1) * width);
        }
        std::vector<uint8_t> z = {0x78, 0x01};
        for (size_t pos = 0; pos < raw.size() || pos == 0;) {
            const size_t n = std::min<size_t>(65535, raw.size() - pos);
            const bool last = pos + n >= raw.size();
            z.push_back(last ? 1 : 0);
            z.push_back((uint8_t)(n & 0xFF));
            z.push_back((uint8_t)(n >> 8));
            z.push_back((uint8_t)(~n & 0xFF));
            z.push_back((uint8_t)((~n >> 8) & 0xFF));
            z.insert(z.end(), raw.begin() + pos, raw.begin() + pos + n);
            pos += n;
            if (last) break;
        }
        uint32_t a = 1, b = 0;  // Adler-32 of the raw stream
        for (uint8_t c : raw) {
            a = (a + c) % 65521;
            b = (b + a) % 65521;
        }
        for (int k = 3; k >= 0; k--) z.push_back((uint8_t)(((b << 16) | a) >> (8 * k)));
        FILE *f = std::fopen(path.c_str(), "wb");
        if (!f) return false;
        static const uint8_t sig[8] = {0x89, 'P', 'N', 'G', '\r', '\n', 0x1A, '\n'};
        std::fwrite(sig, 1, 8, f);
        auto be32 = [](std::vector<uint8_t> &v, uint32_t x) {
            for (int k = 3; k >= 0; k--) v.push_back((uint8_t)(x >> (8 * k)));
        };
        auto chunk = [&](const char *tag, const std::vector<uint8_t> &data) {
            std::vector<uint8_t> c;
            be32(c, (uint32_t)data.size());
            c.insert(c.end(), tag, tag + 4);
            c.insert(c.end(), data.begin(), data.end());
            uint32_t crc = 0xFFFFFFFFu;  // CRC-32 over tag + data
            for (size_t i = 4; i < c.size(); i++) {
                crc ^= c[i];
                for (int k = 0; k < 8; k++) crc = (crc >> 1) ^ (0xEDB88320u & (0u - (crc & 1u)));
            }
            be32(c, crc ^ 0xFFFFFFFFu);
            std::fwrite(c.data(), 1, c.size(), f);
        };
        std::vector<uint8_t> ihdr;
        be32(ihdr, (uint32_t)width);
        be32(ihdr, (uint32_t)height);
        ihdr.insert(ihdr.end(), {8, 2, 0, 0, 0});
        chunk("IHDR", ihdr);
        chunk("IDAT", z);
        chunk("IEND", {});
        std::fclose(f);
        return true;
    }
    // Portable float map (no image codec dependency); write_image's divide-by-weight applied.
    bool write_pfm(const std::string &path) const {
        FILE *f = std::fopen(path.c_str(), "wb");
        if (!f) return false;
        std::fprintf(f, "PF\n%d %d\n-1.0\n", width, height);
        for (int y = height - 1; y >= 0; y--)
            for (int x = 0; x < width; x++) {
                float rgb[3];
                pixel(x, y, rgb);
                std::fwrite(rgb, sizeof(float), 3, f);
            }
        std::fclose(f);
        return true;
    }
};

// gpu::PathTracer<C> (spp, max_depth, tile_size, ray_clamp, wavefront) — always wavefront here.
class HipPathTracer {
  public:
    int spp = 16, max_depth = 5, tile_size = 256;
    float ray_clamp = 0.0f;   // <= 0: reference CPU semantics (no clamp); > 0: GPU clamp
    HipPathTracer() = default;
    HipPathTracer(int spp_, int max_depth_, int tile_size_, float ray_clamp_)
        : spp(spp_), max_depth(max_depth_), tile_size(tile_size_), ray_clamp(ray_clamp_) {}

    // render(const Scene<C>&, Film<C>*): accumulates every tile of the film
    void render(const HipAccelerator &scene, Film &film) const {
        std::vector<akr_rect> tiles;
        for (int y = 0; y < film.height; y += tile_size)
            for (int x = 0; x < film.width; x += tile_size) tiles.push_back({x, y, x + tile_size, y + tile_size});
        akr_pt_params p{spp, max_depth, ray_clamp, 0};
        check(scene.handle(),
              akr_hip_render(scene.handle(), &p, tiles.data(), (int32_t)tiles.size(), film.radiance.data(),
                             film.weight.data()),
              "render");
    }

    // Multi-GPU in one process (akr_hip_render_node): tile j on accelerators[j % n], one per device,
    // each built from the same scene; the merged film equals render() on one of them.
    void render_node(const std::vector<const HipAccelerator *> &accels, Film &film) const {
        if (accels.empty()) throw std::runtime_error("render_node: no accelerators");
        std::vector<akr_rect> tiles;
        for (int y = 0; y < film.height; y += tile_size)
            for (int x = 0; x < film.width; x += tile_size) tiles.push_back({x, y, x + tile_size, y + tile_size});
        std::vector<akr_hip_ctx *> h;
        for (auto *a : accels) h.push_back(a->handle());
        akr_pt_params p{spp, max_depth, ray_clamp, 0};
        check(h[0],
              akr_hip_render_node(h.data(), (int32_t)h.size(), &p, tiles.data(), (int32_t)tiles.size(),
                                  film.radiance.data(), film.weight.data()),
              "render_node");
    }
};

// cpu::AmbientOcclusion<C> (spp, occlude; kernel/integrators/cpu/integrator.h:35-45), rendered on
// the GPU through akr_hip_render_ao.
class HipAmbientOcclusion {
  public:
    int spp = 16, tile_size = 16;
    float occlude = std::numeric_limits<float>::infinity();
    HipAmbientOcclusion() = default;
    HipAmbientOcclusion(int spp_, float occlude_) : spp(spp_), occlude(occlude_) {}

    void render(const HipAccelerator &scene, Film &film) const {
        const int ts = std::max(16, tile_size);  // one call renders every tile: size is a batching knob
        std::vector<akr_rect> tiles;
        for (int y = 0; y < film.height; y += ts)
            for (int x = 0; x < film.width; x += ts) tiles.push_back({x, y, x + ts, y + ts});
        akr_ao_params p{spp, occlude, 0, 0};
        check(scene.handle(),
              akr_hip_render_ao(scene.handle(), &p, tiles.data(), (int32_t)tiles.size(), film.radiance.data(),
                                film.weight.data()),
              "render_ao");
    }
};

}  // namespace akari::hip
