'use strict';
/**
 * Camera of the reference (apps/frontend/src/graphics-core/Camera.ts): same fields, same
 * methods, same math (wgpu-matrix storage semantics via ./wgpu_math).
 */
const { vec3, quat, mat4 } = require('./wgpu_math');

class Camera {
  constructor(Width, Height, InLocation = vec3.fromValues(0, 0, 1), InRollDegree = 0, InPitchDegree = 0,
    InYawDegree = 0, InFOVDegree = 60, InNear = 0.1, InFar = 1000) {
    this.Location = InLocation;                                     // Camera.ts:19-45
    this.Roll = (InRollDegree * Math.PI) / 180.0;
    this.Pitch = (InPitchDegree * Math.PI) / 180.0;
    this.Yaw = (InYawDegree * Math.PI) / 180.0;
    this.AspectRatio = Width / Height;
    this.FOV = (InFOVDegree * Math.PI) / 180.0;
    this.Near = InNear;
    this.Far = InFar;
    this.ProjectionMatrix = this.computeProjectionMatrix();
  }

  GetViewProjectionMatrix() {                                        // Camera.ts:47-53
    return mat4.multiply(this.ProjectionMatrix, this.GetViewMatrix());
  }

  GetViewMatrix() {                                                  // Camera.ts:55-64
    const T = mat4.translation(this.Location);
    const R = mat4.fromQuat(quat.fromEuler(this.Pitch, this.Yaw, this.Roll, 'yxz'));
    return mat4.invert(mat4.multiply(T, R));
  }

  GetForwardVector() {                                               // Camera.ts:66-73
    const q = quat.fromEuler(this.Pitch, this.Yaw, this.Roll, 'yxz');
    return vec3.normalize(vec3.transformQuat(vec3.fromValues(0, 0, -1), q));
  }

  GetRightVector() {                                                 // Camera.ts:75-81
    return vec3.cross(this.GetForwardVector(), vec3.fromValues(0, 1, 0));
  }

  GetLocation() { return this.Location; }
  SetPitch(deg) { this.Pitch = Math.min(Math.PI, Math.max(-Math.PI, (deg * Math.PI) / 180.0)); }
  SetYaw(deg) { this.Yaw = ((deg * Math.PI) / 180.0) % (2 * Math.PI); }
  GetPitch() { return (this.Pitch * 180.0) / Math.PI; }
  GetYaw() { return (this.Yaw * 180.0) / Math.PI; }
  AddPitch(d) { this.Pitch = Math.min(Math.PI / 2, Math.max(-Math.PI / 2, this.Pitch + (d * Math.PI) / 180.0)); }
  AddYaw(d) { this.Yaw = (this.Yaw + (d * Math.PI) / 180.0) % (2 * Math.PI); }
  SetLocation(v) { this.Location = v; }
  AddLocationOffset(o) {
    this.Location[0] += o[0];
    this.Location[1] += o[1];
    this.Location[2] += o[2];
  }
  SetLocationFromXYZ(X, Y, Z) {
    this.Location[0] = X;
    this.Location[1] = Y;
    this.Location[2] = Z;
  }
  SetAspectRatio(W, H) {
    this.AspectRatio = W / H;
    this.ProjectionMatrix = this.computeProjectionMatrix();
  }
  computeProjectionMatrix() {                                        // Camera.ts:165-168
    return mat4.perspective(this.FOV, this.AspectRatio, this.Near, this.Far);
  }
}

module.exports = { Camera };
