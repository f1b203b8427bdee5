// pt_viewer.cpp -- the reference's interactive loop without its window (include/pt_viewer.h).
//
// State and arithmetic follow ogl_path_trace.h (file:line below).  The camera vectors are
// glm::vec4 of float there; glm's generic (non-SIMD) code paths are assumed (glm is not
// vendored and its version is unpinned):
//   dot(vec4 a, b)      = (a.x*b.x + a.y*b.y) + (a.z*b.z + a.w*b.w)
//   normalize(vec4 v)   = v * (1.0f / sqrt(dot(v, v)))
//   cross(vec3 x, y)    = (x.y*y.z - y.y*x.z, x.z*y.x - y.z*x.x, x.x*y.y - y.x*x.y)
//   radians(double d)   = d * 0.01745329251994329576923690768489
// The cursor callback mixes float and double exactly as the C++ source does: products of
// float components stay float (sqrt / atan2 of float arguments are the float overloads),
// everything assigned to a double is computed in double.  Host libm provides sqrtf /
// atan2f / atan2 / sin / cos (the reference links the MSVC CRT: last-ulp differences of
// atan2f / sin / cos there are not pinned by any reference test).
#include "../../include/pt_viewer.h"

#include <cmath>
#include <new>

namespace {

struct Vec4 { float x, y, z, w; };

Vec4 v4(float x, float y, float z, float w) { Vec4 r; r.x = x; r.y = y; r.z = z; r.w = w; return r; }
Vec4 operator+(Vec4 a, Vec4 b) { return v4(a.x + b.x, a.y + b.y, a.z + b.z, a.w + b.w); }
Vec4 operator-(Vec4 a, Vec4 b) { return v4(a.x - b.x, a.y - b.y, a.z - b.z, a.w - b.w); }
Vec4 operator*(Vec4 a, float s) { return v4(a.x * s, a.y * s, a.z * s, a.w * s); }
float dot4(Vec4 a, Vec4 b) { return (a.x * b.x + a.y * b.y) + (a.z * b.z + a.w * b.w); }
Vec4 normalize4(Vec4 v) { return v * (1.0f / std::sqrt(dot4(v, v))); }

const float kPi = 3.141592f;                                   // ogl_path_trace.h:38
const double kRadPerDeg = 0.01745329251994329576923690768489;  // glm::radians

}  // namespace

struct pt_viewer {
    Vec4 position, direction;                   // :53-54
    float move_speed = 10.0f, rot_speed = 0.1f; // :56-57
    bool mF = false, mB = false, mL = false, mR = false, mU = false, mD = false, mC = false;   // :59
    double pxpos = 0.0, pypos = 0.0;            // :60
    int display_mode = 1;                       // :64
    int user_accumulate = 1;                    // :65
    int accumulate = 0;                         // :66
    int frame_count = 0;                        // :162
    float delta_time = 0.0f, last_frame_time = 0.0f;   // :49-50
    bool started = false, close = false;
};

extern "C" {

int pt_viewer_create(const float camera[12], int display_mode, pt_viewer** out) {
    if (!out) return PT_E_ARG;
    *out = nullptr;
    if (display_mode < 1 || display_mode > 4) return PT_E_ARG;
    pt_viewer* v = new (std::nothrow) pt_viewer();
    if (!v) return PT_E_ARG;
    if (camera) {
        v->position = v4(camera[0], camera[1], camera[2], camera[3]);
        v->direction = v4(camera[4], camera[5], camera[6], camera[7]);
    } else {
        v->position = v4(0.0f, -6.0f, 1.0f, 0.0f);
        v->direction = v4(0.0f, 1.0f, 0.0f, 0.0f);
    }
    v->display_mode = display_mode;
    *out = v;
    return PT_OK;
}

void pt_viewer_destroy(pt_viewer* v) { delete v; }

int pt_viewer_set_params(pt_viewer* v, float move_speed, float rot_speed, int user_accumulate) {
    if (!v || (user_accumulate != 0 && user_accumulate != 1)) return PT_E_ARG;
    v->move_speed = move_speed;
    v->rot_speed = rot_speed;
    v->user_accumulate = user_accumulate;
    return PT_OK;
}

// handleMovementInput (:258-299): keys 1-4 pick the display mode on any action (a change
// restarts accumulation); W/A/S/D/Space/LeftShift hold a motion flag from press to release;
// Escape closes the window.
int pt_viewer_key(pt_viewer* v, int key, int action) {
    if (!v) return PT_E_ARG;
    const int prev = v->display_mode;
    if (key >= PT_KEY_1 && key <= PT_KEY_4) v->display_mode = key - PT_KEY_1 + 1;
    if (prev != v->display_mode) v->mC = true;
    bool* flag = nullptr;
    switch (key) {
        case PT_KEY_W: flag = &v->mF; break;
        case PT_KEY_A: flag = &v->mL; break;
        case PT_KEY_S: flag = &v->mB; break;
        case PT_KEY_D: flag = &v->mR; break;
        case PT_KEY_SPACE: flag = &v->mU; break;
        case PT_KEY_LEFT_SHIFT: flag = &v->mD; break;
        default: break;
    }
    if (flag && action == PT_PRESS) *flag = true;
    if (flag && action == PT_RELEASE) *flag = false;
    if (key == PT_KEY_ESCAPE) v->close = true;
    return PT_OK;
}

// cursorPosCallback (:332-364): yaw about z by the x motion, pitch by the y motion, the
// pitch kept inside (-pi/2, pi/2) by refusing the step; the direction keeps its length.
int pt_viewer_cursor(pt_viewer* v, double xpos, double ypos) {
    if (!v) return PT_E_ARG;
    v->mC = true;
    const Vec4 d = v->direction;
    const double yaw_step = ((v->pxpos - xpos) * kRadPerDeg) * (double)v->rot_speed;
    const double pitch_step = ((v->pypos - ypos) * kRadPerDeg) * (double)v->rot_speed;
    const double xy_len = (double)std::sqrt(d.x * d.x + d.y * d.y);     // float expression
    const double yaw = (double)std::atan2(d.y, d.x);                      // float overload
    const double new_yaw = yaw + yaw_step;
    const double len = (double)std::sqrt(d.x * d.x + d.y * d.y + d.z * d.z);
    const double pitch = std::atan2((double)d.z, xy_len);                 // (float, double) -> double
    double new_pitch = pitch + pitch_step;
    if (new_pitch > (double)kPi / 2.0 || new_pitch < (double)(-kPi) / 2.0) new_pitch = pitch;
    const double nz = len * std::sin(new_pitch);
    const double nxy = len * std::cos(new_pitch);
    const double nx = nxy * std::cos(new_yaw);
    const double ny = nxy * std::sin(new_yaw);
    v->direction = v4((float)nx, (float)ny, (float)nz, 0.0f);
    v->pxpos = xpos;
    v->pypos = ypos;
    return PT_OK;
}

int pt_viewer_should_close(const pt_viewer* v) { return v && v->close ? 1 : 0; }

int pt_viewer_next(pt_viewer* v, double now, pt_viewer_frame_info* out) {
    if (!v || !out) return PT_E_ARG;
    if (v->started) {                 // tail of the previous iteration (:199-204)
        v->accumulate = v->user_accumulate;
        if (v->mF || v->mR || v->mB || v->mL || v->mU || v->mD || v->mC) {
            v->accumulate = 0;
            v->frame_count = 0;
        }
        v->mC = false;
    }
    v->started = true;
    // updateCameraBuffer (:301-328), with the frame time measured by the previous iteration
    const Vec4 dir = v->direction;
    const Vec4 fwd = normalize4(dir - v4(0.0f, 0.0f, dir.z, 0.0f));
    const float rx = fwd.y * 1.0f - 0.0f * fwd.z, ry = fwd.z * 0.0f - 1.0f * fwd.x, rz = fwd.x * 0.0f - 0.0f * fwd.y;
    const Vec4 right = v4(rx, ry, rz, 0.0f);
    const Vec4 up = v4(0.0f, 0.0f, 1.0f, 0.0f);
    const float ms = v->move_speed, dt = v->delta_time;
    if (v->mF) v->position = v->position + fwd * ms * dt;
    if (v->mL) v->position = v->position - right * ms * dt;
    if (v->mB) v->position = v->position - fwd * ms * dt;
    if (v->mR) v->position = v->position + right * ms * dt;
    if (v->mU) v->position = v->position + up * ms * dt;
    if (v->mD) v->position = v->position - up * ms * dt;
    v->frame_count++;                                      // :164
    const float current = (float)now;                     // :166-168
    v->delta_time = current - v->last_frame_time;
    v->last_frame_time = current;
    const float cam[12] = {v->position.x, v->position.y, v->position.z, v->position.w,
                           v->direction.x, v->direction.y, v->direction.z, v->direction.w, 0, 0, 0, 0};
    for (int i = 0; i < 12; i++) out->camera[i] = cam[i];
    out->frame = v->frame_count;
    out->accumulate = v->accumulate;
    out->display_mode = v->display_mode;
    out->should_close = v->close ? 1 : 0;
    return PT_OK;
}

int pt_viewer_frame(pt_viewer* v, pt_ctx* ctx, double now, pt_viewer_frame_info* out) {
    if (!v || !ctx) return PT_E_ARG;
    pt_viewer_frame_info info;
    int rc = pt_viewer_next(v, now, &info);
    if (!rc) rc = pt_set_display_mode(ctx, info.display_mode);
    if (!rc) rc = pt_set_camera(ctx, info.camera);
    // enqueued like glDispatchCompute (ogl_path_trace.h:183): the host goes on to the next
    // iteration while the GPU renders; readbacks and pt_sync wait for the frame
    if (!rc) rc = pt_render_async(ctx, info.frame, 1, info.accumulate);
    if (out) *out = info;
    return rc;
}

}  // extern "C"
