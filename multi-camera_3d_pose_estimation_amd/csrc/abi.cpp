// C-ABI plumbing of libmvpose.so: version, thread-local last error, host helpers.
#include "mvp_common.h"

#include <cmath>
#include <cstring>

namespace mvp {

static thread_local char g_last_error[1024] = "";

void set_error(const char* fmt, ...) {
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(g_last_error, sizeof(g_last_error), fmt, ap);
    va_end(ap);
}

void fail(int code, const char* fmt, ...) {
    char buf[1024];
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(buf, sizeof(buf), fmt, ap);
    va_end(ap);
    throw Error(code, buf);
}

}  // namespace mvp

extern "C" int mvp_abi_version(void) { return MVP_ABI_VERSION; }

extern "C" const char* mvp_last_error(void) { return mvp::g_last_error; }

// P = K·[R|T] with the summation order numpy's small dot uses for 3x3 @ 3x4
// (k = 0, 1, 2 left to right).  Reference: utils.py:1318-1319.
extern "C" int mvp_camera_pack(const double* K, const double* dist5, const double* R,
                               const double* T, double* out) {
    MVP_ABI_BEGIN
    MVP_REQUIRE(K && dist5 && R && T && out, "mvp_camera_pack: null pointer");
    std::memset(out, 0, sizeof(double) * MVP_CAM_DOUBLES);
    std::memcpy(out + 0, K, 9 * sizeof(double));
    std::memcpy(out + 9, dist5, 5 * sizeof(double));
    std::memcpy(out + 14, R, 9 * sizeof(double));
    std::memcpy(out + 23, T, 3 * sizeof(double));
    double Rt[3][4];
    for (int i = 0; i < 3; i++) {
        for (int j = 0; j < 3; j++) Rt[i][j] = R[i * 3 + j];
        Rt[i][3] = T[i];
    }
    for (int i = 0; i < 3; i++)
        for (int j = 0; j < 4; j++) {
            double acc = K[i * 3 + 0] * Rt[0][j];
            acc += K[i * 3 + 1] * Rt[1][j];
            acc += K[i * 3 + 2] * Rt[2][j];
            out[26 + i * 4 + j] = acc;
        }
    MVP_ABI_END
}

// Host helper: does OpenCV's fixed-point warp (WarpAffineInvoker) of an img_h x
// img_w destination through minv (dst -> src, 6 doubles) have a source column
// that depends on x only and a source row that depends on y only?
extern "C" int mvp_warp_is_separable(const double* M, int img_h, int img_w, int* out) {
    MVP_ABI_BEGIN
    MVP_REQUIRE(M && out && img_h > 0 && img_w > 0, "mvp_warp_is_separable: bad arguments");
    int sep = 1;
    const int X00 = (int)std::rint((M[1] * 0 + M[2]) * 1024.0);
    for (int y = 1; y < img_h && sep; y++)
        if ((int)std::rint((M[1] * y + M[2]) * 1024.0) != X00) sep = 0;
    const int b0 = (int)std::rint(M[3] * 0 * 1024.0);
    for (int x = 1; x < img_w && sep; x++)
        if ((int)std::rint(M[3] * x * 1024.0) != b0) sep = 0;
    *out = sep;
    MVP_ABI_END
}
