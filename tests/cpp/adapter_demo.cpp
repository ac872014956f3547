// adapter_demo.cpp — renders the reference's Cornell fixture through the C++ host adapter
// (akari_hip.hpp: HipAccelerator + HipPathTracer + Film), the way a reference-side integration
// would call it.  Usage: adapter_demo <CornellBox-Original.obj.mesh> <out.pfm> <w> <h> <spp> [ao]
// ("ao": HipAmbientOcclusion instead of HipPathTracer)
#include <cstdio>
#include <cstring>
#include <fstream>
#include <vector>

#include "../../akarirender-1_amd/csrc/akari_hip.hpp"

int main(int argc, char **argv) {
    if (argc < 6) return 2;
    // BinaryGeometry::load (core/mesh.cpp:48-85)
    std::ifstream in(argv[1], std::ios::binary);
    char magic[18] = {0};
    in.read(magic, 17);
    if (std::strcmp(magic, "AKARI_BINARY_MESH") != 0) return 3;
    uint64_t nv, nt;
    in.read(reinterpret_cast<char *>(&nv), 8);
    in.read(reinterpret_cast<char *>(&nt), 8);
    std::vector<float> v(3 * nv), n(9 * nt), t(6 * nt);
    std::vector<int32_t> idx(3 * nt), mi(nt);
    in.read(reinterpret_cast<char *>(v.data()), 4 * v.size());
    in.read(reinterpret_cast<char *>(n.data()), 4 * n.size());
    in.read(reinterpret_cast<char *>(t.data()), 4 * t.size());
    in.read(reinterpret_cast<char *>(idx.data()), 4 * idx.size());
    in.read(reinterpret_cast<char *>(mi.data()), 4 * mi.size());

    using namespace akari::hip;
    SceneDesc s;
    auto rgb = [&](float r, float g, float b) {
        akr_texture tx{};
        tx.type = AKR_TEX_CONSTANT;
        tx.value[0] = r; tx.value[1] = g; tx.value[2] = b;
        s.textures.push_back(tx);
        return (int32_t)s.textures.size() - 1;
    };
    auto diffuse = [&](int32_t tex) {
        akr_material m{};
        m.type = AKR_MAT_DIFFUSE;
        m.color = tex;
        s.materials.push_back(m);
        return (int32_t)s.materials.size() - 1;
    };
    // resources/data/cornell_box/cornell_box.akari material values, slot order 0..7
    int32_t grey = rgb(0.725f, 0.71f, 0.68f);
    std::vector<int32_t> slots = {diffuse(rgb(0.63f, 0.065f, 0.05f)), diffuse(rgb(0.14f, 0.45f, 0.091f)),
                                  diffuse(grey), diffuse(grey), diffuse(grey), diffuse(grey), diffuse(grey)};
    akr_material light{};
    light.type = AKR_MAT_EMISSIVE;
    light.color = rgb(17, 12, 4);
    s.materials.push_back(light);
    slots.push_back((int32_t)s.materials.size() - 1);
    MeshView mv;
    mv.vertices = v.data(); mv.n_vertices = nv; mv.indices = idx.data(); mv.normals = n.data();
    mv.texcoords = t.data(); mv.material_indices = mi.data(); mv.n_triangles = nt; mv.material_slots = slots;
    s.meshes.push_back(mv);
    for (int32_t p = 0; p < (int32_t)nt; p++)
        if (mi[p] == 7) s.lights.push_back({0, p});
    s.light_power.assign(s.lights.size(), 1.0f);   // equal weights: both Cornell lights have equal power
    s.camera.position[1] = 1.0f;
    s.camera.position[2] = 9.0f;
    s.camera.fov_deg = 15.0;
    s.camera.resolution[0] = std::atoi(argv[3]);
    s.camera.resolution[1] = std::atoi(argv[4]);

    HipAccelerator accel(0);
    accel.build(s);
    akr_ray r{{0.0f, 1.0f, 0.0f}, 1e-3f, {0.0f, 0.0f, -1.0f}, 1e30f};
    akr_hit h;
    bool hit = accel.intersect(r, &h);
    bool occ = accel.occlude(r);
    Film film(s.camera.resolution[0], s.camera.resolution[1]);
    if (argc > 6 && std::strcmp(argv[6], "ao") == 0) {
        HipAmbientOcclusion ao(std::atoi(argv[5]), std::numeric_limits<float>::infinity());
        ao.render(accel, film);
    } else {
        HipPathTracer pt(std::atoi(argv[5]), 5, 16, 0.0f);
        pt.render(accel, film);
    }
    double sum = 0;
    for (float x : film.radiance) sum += x;
    film.write_pfm(argv[2]);
    std::printf("hit=%d geom=%d prim=%d t=%.6f occluded=%d nodes=%llu sum=%.6f\n", (int)hit, h.geom_id, h.prim_id,
                h.t, (int)occ, (unsigned long long)accel.info().n_nodes, sum);
    return 0;
}
