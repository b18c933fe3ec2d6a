// camera.h — Camera with the reference's interface (CPU/camera.h:11-42,
// GPU/camera.cuh:11-36); a value type converted to rt_camera per frame.
#pragma once

#include "../../include/rtmi.h"
#include "rt_vec.hpp"

namespace rtmi {

class Camera {
   public:
    vec4 position;
    mat4 R;
    float yaw_y = 0.0f;  // CPU engine "yaw"
    float yaw_x = 0.0f;  // GPU engine pitch (uninitialised in GPU/camera.cu:3-7; 0 here)

    explicit Camera(vec4 pos) : position(pos), R(1.0f) {}

    // CPU/camera.cpp:9-25: yaw update, R about y, position = R * position
    void rotate_left(float yaw) { rotate_y(-yaw); }
    void rotate_right(float yaw) { rotate_y(yaw); }
    // GPU/camera.cu:27-45: pitch about x
    void rotate_up(float x) { rotate_x(-x); }
    void rotate_down(float x) { rotate_x(x); }

    // CPU/camera.cpp:27-48: step along the view direction, position = look_at(...) * (0,0,0,1)
    void move_forwards(float distance) { move(distance); }
    void move_backwards(float distance) { move(-distance); }

    vec4 get_position() const { return position; }
    mat4 get_R() const { return R; }
    float get_yaw() const { return yaw_y; }
    void set_position(vec4 p) { position = p; }
    void set_R(const mat4& r) { R = r; }
    void set_yaw(float y) { yaw_y = y; }

    rt_camera to_rt() const {
        rt_camera c;
        c.pos[0] = position.x; c.pos[1] = position.y; c.pos[2] = position.z; c.pos[3] = position.w;
        c.yaw_y = yaw_y;
        c.yaw_x = yaw_x;
        return c;
    }

   private:
    void rotate_y(float a) {
        yaw_y += a;
        R[0] = vec4((float)cos(a), 0, (float)sin(a), 0);
        R[2] = vec4(-(float)sin(a), 0, (float)cos(a), 0);
        position = R * position;
    }
    void rotate_x(float a) {
        yaw_x += a;
        R[0] = vec4(1.f, 0, 0, 0);
        R[1] = vec4(0, (float)cos(a), -(float)sin(a), 0);
        R[2] = vec4(0, (float)sin(a), (float)cos(a), 0);
        position = R * position;
    }
    void move(float d) {
        // look_at(from, 0) * (0,0,0,1) is `from`
        position = vec4(position.x - d * (float)sin(yaw_y), position.y, position.z + d * (float)cos(yaw_y), 1.0f);
    }
};

}  // namespace rtmi
