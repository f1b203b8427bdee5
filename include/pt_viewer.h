/* pt_viewer.h -- headless form of the reference's interactive render loop (SURVEY.md §8(f)
 * row 4): the camera controller and the accumulation-reset rule of run(), without a window.
 *
 *   handleMovementInput (GLFW key callback)     ogl_path_trace.h:258-299  -> pt_viewer_key
 *   cursorPosCallback   (GLFW cursor callback)  ogl_path_trace.h:332-364  -> pt_viewer_cursor
 *   loop head: updateCameraBuffer, frameCount++, deltaTime                 -> pt_viewer_next
 *              (ogl_path_trace.h:160-167, 301-328)
 *   uniforms + glDispatchCompute (:174-186)                                -> pt_viewer_frame
 *   loop tail: accumulate = userDefinedAccumulate, reset on motion (:199-204)
 *
 * A windowing front-end forwards its GLFW callbacks unchanged (key codes and actions are
 * GLFW's) and calls pt_viewer_frame once per displayed frame with glfwGetTime(); a replay
 * tool feeds a recorded event script (ptrace --events).  The loop tail of one iteration is
 * applied at the head of the next, which is equivalent: in the reference nothing happens
 * between the event poll and the tail.  The controller is host arithmetic only (binary32
 * as the reference's glm float math, binary64 where the reference computes in double) and
 * needs no GPU; pt_viewer_frame renders through a pt_ctx (pt_api.h).
 *
 * Return 0 on success, a negative PT_E* code (pt_api.h) otherwise.  Not thread-safe.
 */
#ifndef PT_VIEWER_H
#define PT_VIEWER_H

#include "pt_api.h"

#ifdef __cplusplus
extern "C" {
#endif

/* GLFW key codes and actions the reference's callbacks test (glfw3.h values). */
#define PT_KEY_SPACE 32
#define PT_KEY_1 49
#define PT_KEY_2 50
#define PT_KEY_3 51
#define PT_KEY_4 52
#define PT_KEY_A 65
#define PT_KEY_D 68
#define PT_KEY_S 83
#define PT_KEY_W 87
#define PT_KEY_ESCAPE 256
#define PT_KEY_LEFT_SHIFT 340
#define PT_RELEASE 0
#define PT_PRESS 1
#define PT_REPEAT 2

typedef struct pt_viewer pt_viewer;

/* Parameters of one loop iteration's dispatch. */
typedef struct {
    float camera[12];     /* {position.xyzw, direction.xyzw, 0000}: the camera SSBO (:322) */
    int frame;            /* uniform frame (frameCount after ++, :164) */
    int accumulate;       /* uniform accumulate (:181) */
    int display_mode;     /* uniform displayMode (:182) */
    int should_close;     /* ESC was pressed (glfwWindowShouldClose, :298) */
} pt_viewer_frame_info;

/* camera: 12 floats as above, NULL = the reference default (0,-6,1) looking +y (:53-54).
 * display_mode 1..4 (:64).  moveSpeed 10, rotSpeed 0.1, userDefinedAccumulate 1 (:56-65). */
int pt_viewer_create(const float camera[12], int display_mode, pt_viewer** out);
void pt_viewer_destroy(pt_viewer* v);
/* moveSpeed / rotSpeed (ogl_path_trace.h:56-57) and userDefinedAccumulate (:65, 0 or 1). */
int pt_viewer_set_params(pt_viewer* v, float move_speed, float rot_speed, int user_accumulate);

/* GLFW callbacks. */
int pt_viewer_key(pt_viewer* v, int key, int action);
int pt_viewer_cursor(pt_viewer* v, double xpos, double ypos);
/* 1 once Escape was pressed: the reference's loop condition (:160) then ends the loop
 * before the next frame. */
int pt_viewer_should_close(const pt_viewer* v);

/* One loop iteration's host side: the previous iteration's tail (reset rule), the camera
 * move by the previous frame time, frameCount++, then deltaTime = (float)now - lastFrameTime
 * (glfwGetTime() seconds).  Fills *out with the dispatch parameters. */
int pt_viewer_next(pt_viewer* v, double now, pt_viewer_frame_info* out);
/* pt_viewer_next, then on ctx: display mode, camera, and one dispatch
 * pt_render_async(frame, 1, accumulate) -- enqueued, like glDispatchCompute; a readback or
 * pt_sync waits for it.  out may be NULL. */
int pt_viewer_frame(pt_viewer* v, pt_ctx* ctx, double now, pt_viewer_frame_info* out);

#ifdef __cplusplus
}
#endif
#endif /* PT_VIEWER_H */
