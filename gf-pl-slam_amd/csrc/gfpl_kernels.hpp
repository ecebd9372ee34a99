// gfpl_kernels.hpp — launchers implemented in the k_*.hip translation units.
#pragma once
#include "gfpl_state.hpp"

namespace gfpl {

hipError_t launch_stereo_points(const KParams& p, hipStream_t s);
hipError_t launch_stereo_lines(const KParams& p, hipStream_t s);
hipError_t launch_line_uncertainty(const KParams& p, hipStream_t s);
hipError_t launch_init(const KParams& p, hipStream_t s);
hipError_t launch_knn2(const uint8_t* q, int nq, const uint8_t* t, int nt, int cell, int32_t* idx, float* dist,
                       hipStream_t s);
hipError_t launch_cross_points(const KParams& p, hipStream_t s);
hipError_t launch_cross_lines(const KParams& p, hipStream_t s);
hipError_t launch_line_cut(const KParams& p, hipStream_t s, const hipEvent_t* marks /* [2] or null */);
hipError_t launch_pose(const KParams& p, hipStream_t s, hipEvent_t mark /* or null */);
hipError_t launch_step_bytes(const KParams& p, hipStream_t s);
hipError_t launch_need_kf(const KParams& p, hipStream_t s);
hipError_t launch_curr_frame_is_kf(const KParams& p, const int32_t* mask /* device [B] */, hipStream_t s);

size_t stereo_lines_lds(int cap);

}  // namespace gfpl
