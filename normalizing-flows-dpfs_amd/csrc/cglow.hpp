// cglow.hpp -- the packed parameter layout of the conditional-GLOW measurement
// (nfdpf.pack.cglow_tensors; nf/cglow/modules.py), shared by the forward kernel (cglow.hip)
// and its backward (cglow_bwd.hip).
#pragma once

#include "flows.hpp"

namespace nfdpf {
namespace cg {

constexpr int kE = 192;       // particle / frame encoding (3 x 8 x 8)
constexpr int kXH = 8;        // x_hidden_channels (arguments.py:63)
constexpr int kXS = 16;       // x_hidden_size (arguments.py:64)
constexpr int kC = 12;        // y channels after the squeeze
constexpr int kCh = 6;        // coupling half
constexpr int kYH = 8;        // y_hidden_channels

// ---- packed parameter layout (nfdpf.pack.cglow_tensors), floats, per CondGlowStep ----
// conditioning net (x_Con: three 2x2-stride convs, x_Linear: 8->16->16->OUT)
template <int OUT>
struct Cond {
  static constexpr int c0w = 0, c0b = c0w + kXH * 3 * 4, c2w = c0b + kXH, c2b = c2w + kXH * kXH * 4,
                       c4w = c2b + kXH, c4b = c4w + kXH * kXH * 4, l0w = c4b + kXH, l0b = l0w + kXS * kXH,
                       l2w = l0b + kXS, l2b = l2w + kXS * kXS, l4w = l2b + kXS, l4b = l4w + OUT * kXS,
                       size = l4b + OUT;
};
using CondA = Cond<2 * kC>;    // actnorm: (logs, bias)
using CondI = Cond<kC * kC>;   // 1x1 conv weight
struct Aff {                   // CondAffineCoupling
  static constexpr int r0w = 0, r0b = r0w + 16 * 3 * 9, r2w = r0b + 16, r2b = r2w + kCh * 16 * 4,
                       r4w = r2b + kCh, r4b = r4w + kCh * kCh * 9, f0w = r4b + kCh,
                       f0ab = f0w + kYH * kC * 9, f0al = f0ab + kYH, f2w = f0al + kYH,
                       f2ab = f2w + kYH * kYH, f2al = f2ab + kYH, f4w = f2al + kYH,
                       f4b = f4w + kC * kYH * 9, f4l = f4b + kC, f4nb = f4l + kC, size = f4nb + kC;
};
constexpr int kOffA = 0, kOffI = CondA::size, kOffF = kOffI + CondI::size;
constexpr int kStep = kOffF + Aff::size;

}  // namespace cg
}  // namespace nfdpf
