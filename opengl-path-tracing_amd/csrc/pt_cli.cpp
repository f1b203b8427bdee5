// ptrace -- headless C++ host driver: the reference's main.cpp/run() without the window.
//
//   main.cpp:6-11, ogl_path_trace.h:71-216 (run), :367-530 (setupBuffers)
// The reference ignores argv and hard-codes scene_data/freeobj.txt (absent from the repo,
// SURVEY.md §0.1); this driver honours the README's intent (readme.md:8-9): the .obj and
// .mtl come from the command line.  Frames f = 1..spp are rendered with accumulate = 0
// on frame 1 (ogl_path_trace.h:160-204 after a reset), fused `chunk` frames per launch,
// optionally row-split across several GPUs of this node: --ranks R contexts (rank r on device
// r mod G), the scene validated once and broadcast, the frame gathered over RCCL (pt_group.h).
//
// Output: RGBA32F accumulation as PFM (row 0 = bottom, like the GL texture) and the
// ACES-tonemapped RGBA8 view as binary PPM (screenQuadFrag.c).
#include "../../include/pt_api.h"
#include "../../include/pt_group.h"
#include "../../include/pt_scene.h"
#include "../../include/pt_viewer.h"

#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <sstream>
#include <string>
#include <vector>

static void usage() {
    std::fprintf(stderr,
                 "usage: ptrace <scene.obj> <scene.mtl | -> [--width W] [--height H] [--spp S] [--chunk C]\n"
                 "              [--bounces B] [--mode 1..4] [--gpus G] [--ranks R] [--pfm out.pfm] [--ppm out.ppm]\n"
                 "              [--camera px py pz dx dy dz] [--robust] [--events script.txt]\n"
                 "  --robust  general Wavefront ingest (v/vt/vn corners, polygons, negative indices,\n"
                 "            free-form MTL; '-' as the MTL uses the OBJ's mtllib)\n"
                 "  --events  replay a recorded interactive session instead of --spp frames: the\n"
                 "            reference's render loop with its camera controller and accumulation\n"
                 "            reset (include/pt_viewer.h).  Script lines:\n"
                 "              frame T            one loop iteration at glfwGetTime() = T seconds\n"
                 "              frames N T0 DT     N iterations at T0, T0+DT, ...\n"
                 "              key K ACTION       key callback; K = GLFW code or w a s d 1-4 space shift esc,\n"
                 "                                 ACTION = press | release | repeat\n"
                 "              cursor X Y         cursor callback\n"
                 "            '#' starts a comment; the loop ends early once esc was pressed\n"
                 "  --gpus G        devices 0..G-1 of this node\n"
                 "  --ranks R       row-split contexts (default G; rank r renders rows r, r+R, ... on device\n"
                 "                  r mod G); the frame is gathered over RCCL on device 0\n"
                 "  --checkpoint F  after rendering, save the RGBA32F accumulation and the next frame\n"
                 "                  number (text header 'PTCK2 W H next_frame bounces mode tris nodes' + the\n"
                 "                  camera's 6 floats, then W*H*4 floats)\n"
                 "  --resume F      continue a saved accumulation: frames next_frame.. with accumulate = 1,\n"
                 "                  the same image as one uninterrupted run\n"
                 "  --json          print a JSON summary line\n"
                 "  --gpu-bvh       build the BVH on GPU 0 (pt_bvh_build_gpu; the same nodes)\n");
}

// Checkpoint of a progressive render (SURVEY.md §5 checkpoint / resume): the running mean
// (computeShader.c:548-551) only needs the accumulation image and the next frame number.
// The header also records what the running mean depends on besides the image -- bounces,
// display mode, the scene's triangle and node counts and the camera -- and --resume refuses a
// checkpoint that does not match them (a silent blend of two different renders otherwise).
struct CkptKey {
    int bounces, mode, tris, nodes;
    float cam[6];
};

static bool save_checkpoint(const std::string& path, int W, int H, int next_frame, const CkptKey& key,
                            const std::vector<float>& img) {
    FILE* f = std::fopen(path.c_str(), "wb");
    if (!f) return false;
    std::fprintf(f, "PTCK2 %d %d %d %d %d %d %d %.9g %.9g %.9g %.9g %.9g %.9g\n", W, H, next_frame, key.bounces,
                 key.mode, key.tris, key.nodes, key.cam[0], key.cam[1], key.cam[2], key.cam[3], key.cam[4], key.cam[5]);
    const bool ok = std::fwrite(img.data(), 4, img.size(), f) == img.size();
    return std::fclose(f) == 0 && ok;
}

static bool load_checkpoint(const std::string& path, int W, int H, int& next_frame, CkptKey& key,
                            std::vector<float>& img, std::string& err) {
    FILE* f = std::fopen(path.c_str(), "rb");
    if (!f) { err = "cannot open " + path; return false; }
    int w = 0, h = 0, nf = 0;
    char magic[8] = {0};
    bool ok = std::fscanf(f, "%5s %d %d %d %d %d %d %d %g %g %g %g %g %g", magic, &w, &h, &nf, &key.bounces, &key.mode,
                          &key.tris, &key.nodes, &key.cam[0], &key.cam[1], &key.cam[2], &key.cam[3], &key.cam[4],
                          &key.cam[5]) == 14 &&
              std::string(magic) == "PTCK2" && std::fgetc(f) == '\n';
    if (!ok) err = path + ": not a PTCK2 checkpoint";
    else if (w != W || h != H) { ok = false; err = path + ": checkpoint is " + std::to_string(w) + "x" + std::to_string(h); }
    else if (nf < 1) { ok = false; err = path + ": bad next frame"; }
    if (ok) {
        img.assign(4 * (size_t)W * H, 0.0f);
        ok = std::fread(img.data(), 4, img.size(), f) == img.size();
        if (!ok) err = path + ": truncated";
        next_frame = nf;
    }
    std::fclose(f);
    return ok;
}

// One event of an --events script (see usage()).
struct Event {
    int kind;          // 0 frame, 1 key, 2 cursor
    double a, b;
    int key, action;
};

static bool parse_events(const char* path, std::vector<Event>& ev, std::string& err) {
    std::ifstream in(path);
    if (!in) { err = std::string("cannot open ") + path; return false; }
    std::string line;
    int ln = 0;
    while (std::getline(in, line)) {
        ln++;
        const size_t hash = line.find('#');
        if (hash != std::string::npos) line.resize(hash);
        std::istringstream ss(line);
        std::string op;
        if (!(ss >> op)) continue;
        Event e = {0, 0.0, 0.0, 0, 0};
        bool ok = true;
        if (op == "frame") {
            ok = static_cast<bool>(ss >> e.a);
            ev.push_back(e);
        } else if (op == "frames") {
            long n = 0;
            double t0 = 0, dt = 0;
            ok = static_cast<bool>(ss >> n >> t0 >> dt) && n >= 0 && n <= 10000000;
            for (long i = 0; ok && i < n; i++) { e.a = t0 + (double)i * dt; ev.push_back(e); }
        } else if (op == "key") {
            std::string k, a;
            ok = static_cast<bool>(ss >> k >> a);
            e.kind = 1;
            if (k == "w" || k == "W") e.key = PT_KEY_W;
            else if (k == "a" || k == "A") e.key = PT_KEY_A;
            else if (k == "s" || k == "S") e.key = PT_KEY_S;
            else if (k == "d" || k == "D") e.key = PT_KEY_D;
            else if (k == "space") e.key = PT_KEY_SPACE;
            else if (k == "shift") e.key = PT_KEY_LEFT_SHIFT;
            else if (k == "esc") e.key = PT_KEY_ESCAPE;
            else if (k.size() == 1 && k[0] >= '1' && k[0] <= '4') e.key = PT_KEY_1 + (k[0] - '1');
            else e.key = std::atoi(k.c_str());
            if (a == "press") e.action = PT_PRESS;
            else if (a == "release") e.action = PT_RELEASE;
            else if (a == "repeat") e.action = PT_REPEAT;
            else e.action = std::atoi(a.c_str());
            ev.push_back(e);
        } else if (op == "cursor") {
            e.kind = 2;
            ok = static_cast<bool>(ss >> e.a >> e.b);
            ev.push_back(e);
        } else {
            ok = false;
        }
        if (!ok) { err = std::string(path) + ":" + std::to_string(ln) + ": bad event line"; return false; }
    }
    return true;
}

#define CHECK(expr, ctx)                                                              \
    do {                                                                              \
        int rc_ = (expr);                                                             \
        if (rc_) {                                                                    \
            std::fprintf(stderr, "%s failed (%d): %s\n", #expr, rc_, pt_last_error(ctx)); \
            return 1;                                                                 \
        }                                                                             \
    } while (0)

int main(int argc, char** argv) {
    if (argc < 3) { usage(); return 2; }
    const char* obj = argv[1];
    const char* mtl = argv[2];
    int W = 1000, H = 800, spp = 64, chunk = 16, bounces = 5, mode = 1, gpus = 1, ranks = 0;   // ogl_path_trace.h:45-46
    std::string pfm = "out.pfm", ppm = "out.ppm";
    float cam[12] = {0, -6, 1, 0, 0, 1, 0, 0, 0, 0, 0, 0};                          // ogl_path_trace.h:53-54
    bool robust = false, json = false, gpu_bvh = false;
    const char* events = nullptr;
    std::string checkpoint, resume;
    for (int i = 3; i < argc; i++) {
        std::string a = argv[i];
        auto next = [&](void) -> const char* { if (i + 1 >= argc) { usage(); std::exit(2); } return argv[++i]; };
        if (a == "--width") W = std::atoi(next());
        else if (a == "--height") H = std::atoi(next());
        else if (a == "--spp") spp = std::atoi(next());
        else if (a == "--chunk") chunk = std::atoi(next());
        else if (a == "--bounces") bounces = std::atoi(next());
        else if (a == "--mode") mode = std::atoi(next());
        else if (a == "--gpus") gpus = std::atoi(next());
        else if (a == "--ranks") ranks = std::atoi(next());
        else if (a == "--pfm") pfm = next();
        else if (a == "--ppm") ppm = next();
        else if (a == "--camera") { for (int k = 0; k < 6; k++) cam[k < 3 ? k : k + 1] = (float)std::atof(next()); }
        else if (a == "--robust") robust = true;
        else if (a == "--events") events = next();
        else if (a == "--checkpoint") checkpoint = next();
        else if (a == "--resume") resume = next();
        else if (a == "--json") json = true;
        else if (a == "--gpu-bvh") gpu_bvh = true;
        else { usage(); return 2; }
    }
    if (ranks == 0) ranks = gpus;
    if (spp < 1 || chunk < 1 || gpus < 1 || ranks < 1) { usage(); return 2; }
    if (events && (!resume.empty() || !checkpoint.empty())) {
        std::fprintf(stderr, "--events excludes --resume / --checkpoint\n");
        return 2;
    }
    int first = 1;                        // frame number of the first frame rendered
    std::vector<float> prior;
    CkptKey saved = {};
    if (!resume.empty()) {
        std::string err;
        if (!load_checkpoint(resume, W, H, first, saved, prior, err)) { std::fprintf(stderr, "%s\n", err.c_str()); return 2; }
    }

    auto t0 = std::chrono::steady_clock::now();
    pt_scene* sc = nullptr;
    const bool mtl_from_obj = std::string(mtl) == "-";
    if (mtl_from_obj && !robust) { std::fprintf(stderr, "'-' as the MTL needs --robust\n"); return 2; }
    int rc = pt_scene_load_obj_ex(obj, mtl_from_obj ? nullptr : mtl, robust ? PT_LOAD_ROBUST : PT_LOAD_REFERENCE, &sc);
    if (!rc) rc = pt_scene_add_builtins(sc);
    if (!rc) rc = gpu_bvh ? pt_scene_build_bvh_gpu(sc, 0) : pt_scene_build_bvh(sc);
    if (rc) { std::fprintf(stderr, "scene: %s (%d)\n", pt_scene_last_error(sc), rc); pt_scene_free(sc); return 1; }
    int cnt[5];
    pt_scene_counts(sc, cnt);
    std::vector<float> tris(16 * (size_t)cnt[0]), mats(16 * (size_t)cnt[1]), sph(8 * (size_t)cnt[2]), nodes(12 * (size_t)cnt[3]);
    pt_scene_get_tris(sc, tris.data(), cnt[0]);
    pt_scene_get_mats(sc, mats.data(), cnt[1]);
    pt_scene_get_spheres(sc, sph.data(), cnt[2]);
    pt_scene_get_nodes(sc, nodes.data(), cnt[3]);
    pt_scene_free(sc);
    double t_scene = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
    std::printf("# of polygons: %d  # of materials: %d (+5 built-in)  # of spheres: %d  BVH nodes: %d  (%.3f s)\n",
                cnt[0], cnt[4], cnt[2], cnt[3], t_scene);
    const CkptKey key = {bounces, mode, cnt[0], cnt[3], {cam[0], cam[1], cam[2], cam[4], cam[5], cam[6]}};
    if (!resume.empty() &&
        (saved.bounces != key.bounces || saved.mode != key.mode || saved.tris != key.tris || saved.nodes != key.nodes ||
         std::memcmp(saved.cam, key.cam, sizeof(key.cam)) != 0)) {
        std::fprintf(stderr, "%s: checkpoint of a different render (bounces %d mode %d tris %d nodes %d camera "
                             "%g %g %g %g %g %g); refusing to blend\n", resume.c_str(), saved.bounces, saved.mode,
                     saved.tris, saved.nodes, saved.cam[0], saved.cam[1], saved.cam[2], saved.cam[3], saved.cam[4],
                     saved.cam[5]);
        return 2;
    }

    const int nctx = ranks;
    std::vector<pt_ctx*> ctx(nctx, nullptr);
    for (int g = 0; g < nctx; g++) {
        pt_config cfg = {W, H, bounces, mode, 0, 1, g % gpus, g, nctx};
        CHECK(pt_create(&cfg, &ctx[g]), ctx[g]);
    }
    pt_group* group = nullptr;
    if (nctx > 1) {   // one RCCL communicator over the devices; the scene is validated once
        int grc = pt_group_create(ctx.data(), nctx, &group);
        if (!grc) grc = pt_group_upload_scene(group, tris.data(), cnt[0], nodes.data(), cnt[3], mats.data(), cnt[1],
                                              sph.data(), cnt[2]);
        if (grc) { std::fprintf(stderr, "pt_group: %s (%d)\n", pt_group_last_error(group), grc); return 1; }
    }
    for (int g = 0; g < nctx; g++) {
        if (!group)
            CHECK(pt_upload_scene(ctx[g], tris.data(), cnt[0], nodes.data(), cnt[3], mats.data(), cnt[1], sph.data(), cnt[2]), ctx[g]);
        CHECK(pt_set_camera(ctx[g], cam), ctx[g]);
        if (!prior.empty()) {             // this context's rows of the saved image
            int rows = 0, r0 = 0, rs = 1;
            pt_rows(ctx[g], &rows, &r0, &rs);
            std::vector<float> part(4 * (size_t)rows * W);
            for (int k = 0; k < rows; k++)
                std::memcpy(&part[4 * (size_t)k * W], &prior[4 * (size_t)(r0 + k * rs) * W], 16 * (size_t)W);
            CHECK(pt_write_rgba32f(ctx[g], part.data(), part.size() * 4), ctx[g]);
        }
    }
    auto t1 = std::chrono::steady_clock::now();
    int frames_run = 0, resets = 0;
    if (events) {
        // the reference's render loop (ogl_path_trace.h:160-204) driven by a recorded session
        std::vector<Event> ev;
        std::string err;
        if (!parse_events(events, ev, err)) { std::fprintf(stderr, "%s\n", err.c_str()); return 2; }
        pt_viewer* view = nullptr;
        if (pt_viewer_create(cam, mode, &view)) { std::fprintf(stderr, "pt_viewer_create failed\n"); return 1; }
        for (const Event& e : ev) {
            if (e.kind == 1) pt_viewer_key(view, e.key, e.action);
            else if (e.kind == 2) pt_viewer_cursor(view, e.a, e.b);
            else {
                if (pt_viewer_should_close(view)) break;     // glfwWindowShouldClose (:160)
                pt_viewer_frame_info fi;
                pt_viewer_next(view, e.a, &fi);
                for (int g = 0; g < nctx; g++) {
                    CHECK(pt_set_display_mode(ctx[g], fi.display_mode), ctx[g]);
                    CHECK(pt_set_camera(ctx[g], fi.camera), ctx[g]);
                    CHECK(pt_render_async(ctx[g], fi.frame, 1, fi.accumulate), ctx[g]);
                }
                frames_run++;
                resets += fi.accumulate == 0;
            }
        }
        pt_viewer_destroy(view);
        spp = frames_run;
    } else {
        for (int k = 0; k < spp; k += chunk) {
            const int n = std::min(chunk, spp - k), f0 = first + k;
            // frame 1 after a reset overwrites (accumulate = 0); a resumed run accumulates
            for (int g = 0; g < nctx; g++) CHECK(pt_render_async(ctx[g], f0, n, f0 == 1 ? 0 : 1), ctx[g]);
        }
    }
    std::vector<float> img(4 * (size_t)W * H, 0.0f);
    double gather_ms = 0.0;
    if (group) {      // stream-ordered after every context's renders: the gather is the sync
        int grc = pt_group_gather_rgba32f(group, img.data(), img.size() * 4, 0);
        if (grc) { std::fprintf(stderr, "pt_group_gather_rgba32f: %s (%d)\n", pt_group_last_error(group), grc); return 1; }
        pt_group_stats(group, &gather_ms, nullptr);
    }
    for (int g = 0; g < nctx; g++) CHECK(pt_sync(ctx[g]), ctx[g]);
    double secs = std::chrono::duration<double>(std::chrono::steady_clock::now() - t1).count();
    if (events) std::printf("replayed %s: %d frames, %d accumulation restarts\n", events, frames_run, resets);

    std::vector<unsigned char> rgba(4 * (size_t)W * H, 0);
    if (group) {      // the ACES view of the gathered frame, tonemapped on the root device
        int grc = pt_group_gather_rgba8_aces(group, rgba.data(), rgba.size(), 0);
        if (grc) { std::fprintf(stderr, "pt_group_gather_rgba8_aces: %s (%d)\n", pt_group_last_error(group), grc); return 1; }
    }
    for (int g = 0; g < nctx && !group; g++) {     // one context: its own ACES view and rows
        int rows = 0, r0 = 0, rs = 1;
        pt_rows(ctx[g], &rows, &r0, &rs);
        std::vector<unsigned char> part8(4 * (size_t)rows * W);
        CHECK(pt_read_rgba8_aces(ctx[g], part8.data(), part8.size()), ctx[g]);
        CHECK(pt_read_rgba32f(ctx[g], img.data(), img.size() * 4), ctx[g]);
        for (int k = 0; k < rows; k++)
            std::memcpy(&rgba[4 * (size_t)(r0 + k * rs) * W], &part8[4 * (size_t)k * W], 4 * (size_t)W);
    }
    pt_group_destroy(group);
    for (int g = 0; g < nctx; g++) pt_destroy(ctx[g]);
    std::printf("rendered %dx%d, %d spp, %d bounces on %d GPU(s), %d context(s): %.3f s, %.3f ms/frame\n", W, H, spp,
                bounces, gpus, nctx, secs, secs * 1e3 / (spp > 0 ? spp : 1));
    if (group) std::printf("RCCL gather: %.3f ms\n", gather_ms);
    if (!checkpoint.empty()) {
        if (!save_checkpoint(checkpoint, W, H, first + spp, key, img)) {
            std::fprintf(stderr, "cannot write checkpoint %s\n", checkpoint.c_str());
            return 1;
        }
    }
    if (json)
        std::printf("{\"width\": %d, \"height\": %d, \"frames\": %d, \"first_frame\": %d, \"bounces\": %d, "
                    "\"gpus\": %d, \"contexts\": %d, \"seconds\": %.6f, \"ms_per_frame\": %.4f, \"triangles\": %d, "
                    "\"nodes\": %d, \"gather_ms\": %.4f}\n",
                    W, H, spp, first, bounces, gpus, nctx, secs, secs * 1e3 / (spp > 0 ? spp : 1), cnt[0], cnt[3],
                    gather_ms);

    if (FILE* f = std::fopen(pfm.c_str(), "wb")) {       // PFM rows run bottom-to-top: no flip
        std::fprintf(f, "PF\n%d %d\n-1.0\n", W, H);
        for (size_t i = 0; i < (size_t)W * H; i++) std::fwrite(&img[4 * i], 4, 3, f);
        std::fclose(f);
    }
    if (FILE* f = std::fopen(ppm.c_str(), "wb")) {       // PPM rows run top-to-bottom: flip
        std::fprintf(f, "P6\n%d %d\n255\n", W, H);
        for (int y = H - 1; y >= 0; y--)
            for (int x = 0; x < W; x++) std::fwrite(&rgba[4 * ((size_t)y * W + x)], 1, 3, f);
        std::fclose(f);
    }
    return 0;
}
