// The LDS-DMA conv / GEMM launchers (igemm.h run_glds_part): included only by the family translation units
// glds_p0..3.hip and glds_x3.hip, each instantiating its family once.
#pragma once

#include <algorithm>
#include <tuple>
#include <type_traits>

#include "igemm.h"

namespace tony {
namespace glds {

template <bool XF, int PART>
int run_glds_part(const Gather& g, const void* B, int64_t ldb, void* C, int64_t ldc, int64_t M, int64_t N, int epi,
                  float* st, int64_t sstride, int v, hipStream_t stream, RowMap rmap, BTaps bt, int stream_m,
                  X3Planes xp, const MultiClass* classes) {
  constexpr bool x3 = XF;
  const GldsVariant gv = x3 ? GldsVariant{kX3Variants[v - kX3First].bm, kX3Variants[v - kX3First].cap,
                                          kX3Variants[v - kX3First].stages, kX3Variants[v - kX3First].kb,
                                          kX3Variants[v - kX3First].nwm}
                            : kGldsVariants[v - kGldsFirst];
  const int64_t bn = pick_bn(N, gv.cap);
  using std::integral_constant;
  const auto launch = [&](auto bm, auto bnc, auto st_, auto kb, auto nwm, auto il, auto x3c, auto pfc) -> int {
    constexpr int BM = decltype(bm)::value, BN = decltype(bnc)::value, ST = decltype(st_)::value;
    constexpr int KB = decltype(kb)::value, NWM = decltype(nwm)::value;
    constexpr bool IL = decltype(il)::value, X3 = decltype(x3c)::value;
    constexpr bool PF = decltype(pfc)::value > 0 && decltype(pfc)::value < 2;  // 1: fragment prefetch
    constexpr int WPE = decltype(pfc)::value >= 2 ? decltype(pfc)::value : 0;  // >= 2: waves per SIMD
    constexpr int PL = X3 ? 2 : 1;
    if constexpr (BN % (64 / (KB / 8)) != 0 || BM * (BN + 8) > ST * PL * (BM + BN) * KB ||
                  ST * PL * (BM + BN) * KB * 2 > 163840 || (X3 && IL) || (PF && (X3 || IL)) ||
                  (WPE > 0 && (X3 || ST * (BM + BN) * KB * 2 * (WPE * 4 / (2 * NWM)) > 163840))) {
      return -3;
    } else {
      const int tiles_n = ceil_div(N, BN);
      MultiClass mc{};
      int64_t tiles = 0;
      if (classes != nullptr) {  // the classes' tile ranges end to end (M is unused then)
        mc = *classes;
        for (int i = 0; i < mc.n; ++i) {
          if (mc.c[i].g.Cs % KB != 0 || mc.c[i].bt.S == 0) return -3;  // uniform-tap class taps only
          const int64_t t = static_cast<int64_t>(ceil_div(mc.c[i].M, BM)) * tiles_n;
          if (tiles + t + 8 > 0x7fffffff) return -2;
          mc.c[i].begin = static_cast<int>(tiles);
          mc.c[i].tiles = static_cast<int>(t);
          tiles += (t + 7) & ~int64_t{7};
        }
      } else {
        tiles = static_cast<int64_t>(ceil_div(M, BM)) * tiles_n;
      }
      if (tiles > 0x7fffffff) return -2;
      SplitK sk{};
      int grid = static_cast<int>(tiles);
      if (stream_m > 0) {
        // worth it while the tiles leave CUs idle or a near-empty last wave: a few tiles per CU at most
        const int cus = num_cus_of_current();
        const int64_t iters = tiles * ((g.K + KB - 1) / KB);
        int64_t G = static_cast<int64_t>(stream_m) * cus;
        G = std::min<int64_t>(G, iters / 4);  // >= 4 K-steps per workgroup
        if (tiles > 4 * G || tiles > kStreamMaxTiles || G < 2 || tiles % G == 0) return -3;
        const SplitWs& ws = splitk_ws();
        if (ws.slab != nullptr && ws.cnt != nullptr && ws.ncnt >= 2 * tiles &&
            ws.slab_floats >= 2 * G * BM * BN) {
          sk.slab = ws.slab;
          sk.cnt = ws.cnt;
          sk.ntiles = static_cast<int>(tiles);
          sk.stream = 1;
          grid = static_cast<int>(G);
        }
      }
      const auto args = std::make_tuple(g, static_cast<const uint16_t*>(B), ldb, static_cast<uint16_t*>(C), ldc,
                                        static_cast<int>(M), static_cast<int>(N), st, sstride, epi, tiles_n, rmap, bt,
                                        sk, xp, mc);
      // the lean kernels (FT 0) unless this launch runs stream-K (1) or the residue classes (2)
      const int ft = classes != nullptr ? 2 : (sk.stream != 0 ? 1 : 0);
      const auto go = [&](auto kern) { std::apply([&](auto... a) { kern<<<grid, 128 * NWM, 0, stream>>>(a...); }, args); };
      if (xp.atab != nullptr) {  // the BN-apply-on-load prototype: one tile family
        if constexpr (!X3 && !IL && !PF && WPE == 0 && BM == 128 && ST == 3 && KB == 32 && NWM == 2 && BN <= 128) {
          if (g.Cs % KB != 0 || g.R != 1 || g.S != 1 || ft) return -3;
          go(conv_glds_kernel<BM, BN, ST, KB, true, NWM, false, false, true>);
          TONY_LAUNCH_CHECK();
          return 0;
        } else {
          return -3;
        }
      }
      if constexpr (X3) {
        if (g.Cs % KB != 0) return -3;  // the fused planes run the uniform-tap loop only
        if (ft == 1)
          go(conv_glds_kernel<BM, BN, ST, KB, true, NWM, false, true, false, false, 1>);
        else if (ft == 0)
          go(conv_glds_kernel<BM, BN, ST, KB, true, NWM, false, true, false, false, 0>);
        else
          return -3;
      } else if (g.Cs % KB == 0 && glds_uni_enabled()) {
        if constexpr (WPE > 0) {
          if (ft == 1)
            go(conv_glds_occ_kernel<BM, BN, ST, KB, true, NWM, IL, WPE, 1>);
          else if (ft == 2)
            go(conv_glds_occ_kernel<BM, BN, ST, KB, true, NWM, IL, WPE, 2>);
          else
            go(conv_glds_occ_kernel<BM, BN, ST, KB, true, NWM, IL, WPE, 0>);
        } else {
          if (ft == 1)
            go(conv_glds_kernel<BM, BN, ST, KB, true, NWM, IL, false, false, PF, 1>);
          else if (ft == 2)
            go(conv_glds_kernel<BM, BN, ST, KB, true, NWM, IL, false, false, PF, 2>);
          else
            go(conv_glds_kernel<BM, BN, ST, KB, true, NWM, IL, false, false, PF, 0>);
        }
      } else if (IL || bt.S != 0) {
        return -3;  // the interleaved form and the class taps exist for the uniform-tap loop only
      } else if constexpr (IL) {
        return -3;  // (no general-loop instance in the interleaved family: it is the plain family's)
      } else {
        if (ft == 2) return -3;  // (the residue classes are uniform-tap only)
        if constexpr (WPE > 0) {
          if (ft == 1)
            go(conv_glds_occ_kernel<BM, BN, ST, KB, false, NWM, false, WPE, 1>);
          else
            go(conv_glds_occ_kernel<BM, BN, ST, KB, false, NWM, false, WPE, 0>);
        } else {
          if (ft == 1)
            go(conv_glds_kernel<BM, BN, ST, KB, false, NWM, false, false, false, PF, 1>);
          else
            go(conv_glds_kernel<BM, BN, ST, KB, false, NWM, false, false, false, PF, 0>);
        }
      }
      TONY_LAUNCH_CHECK();
      return 0;
    }
  };
  const auto by_bn = [&](auto bm, auto st_, auto kb, auto cap, auto nwm, auto il, auto x3c, auto pfc) -> int {
    constexpr int CAP = decltype(cap)::value;
    switch (bn) {
      case 32: return launch(bm, integral_constant<int, 32>{}, st_, kb, nwm, il, x3c, pfc);
      case 64: return launch(bm, integral_constant<int, 64>{}, st_, kb, nwm, il, x3c, pfc);
      case 96: return launch(bm, integral_constant<int, 96>{}, st_, kb, nwm, il, x3c, pfc);
      case 128: return launch(bm, integral_constant<int, 128>{}, st_, kb, nwm, il, x3c, pfc);
      case 160:
        if constexpr (CAP >= 160) return launch(bm, integral_constant<int, 160>{}, st_, kb, nwm, il, x3c, pfc);
        break;
      case 192:
        if constexpr (CAP >= 192) return launch(bm, integral_constant<int, 192>{}, st_, kb, nwm, il, x3c, pfc);
        break;
      default: break;
    }
    return -3;
  };
  using I2 = integral_constant<int, 2>;
  using I3 = integral_constant<int, 3>;
  using I4 = integral_constant<int, 4>;
  using K32 = integral_constant<int, 32>;
  using K64 = integral_constant<int, 64>;
  using M64 = integral_constant<int, 64>;
  using M128 = integral_constant<int, 128>;
  using C128 = integral_constant<int, 128>;
  using C192 = integral_constant<int, 192>;
  using M256 = integral_constant<int, 256>;
  using I5 = integral_constant<int, 5>;
  using W2 = integral_constant<int, 2>;
  using W4 = integral_constant<int, 4>;
  using NO = std::false_type;
  using ILV = std::true_type;
  using WP2 = integral_constant<int, 2>;  // (the last by_bn argument: 0 plain, 1 fragment prefetch, >= 2
  using WP3 = integral_constant<int, 3>;  //  waves per SIMD of conv_glds_occ_kernel)
  using WP4 = integral_constant<int, 4>;
  if constexpr (XF) {
    using X = std::true_type;
    switch (v - kX3First) {
      case 0: return by_bn(M256{}, I2{}, K32{}, C128{}, W4{}, NO{}, X{}, NO{});
      case 1: return by_bn(M128{}, I3{}, K32{}, C192{}, W2{}, NO{}, X{}, NO{});
      case 2: return by_bn(M128{}, I4{}, K32{}, C128{}, W2{}, NO{}, X{}, NO{});
      case 3: return by_bn(M128{}, I2{}, K64{}, C128{}, W2{}, NO{}, X{}, NO{});
      case 4: return by_bn(M256{}, I3{}, K32{}, C128{}, W4{}, NO{}, X{}, NO{});
      case 5: return by_bn(M64{}, I4{}, K32{}, C128{}, W2{}, NO{}, X{}, NO{});
      default: return -3;
    }
  } else {
  switch (v - kGldsFirst) {
    case 0: if constexpr (glds_part(0) == PART) { return by_bn(M128{}, I2{}, K64{}, C128{}, W2{}, NO{}, NO{}, NO{}); } return -3;
    case 1: if constexpr (glds_part(1) == PART) { return by_bn(M128{}, I3{}, K32{}, C128{}, W2{}, NO{}, NO{}, NO{}); } return -3;
    case 2: if constexpr (glds_part(2) == PART) { return by_bn(M128{}, I4{}, K32{}, C128{}, W2{}, NO{}, NO{}, NO{}); } return -3;
    case 3: if constexpr (glds_part(3) == PART) { return by_bn(M128{}, I3{}, K32{}, C192{}, W2{}, NO{}, NO{}, NO{}); } return -3;
    case 4: if constexpr (glds_part(4) == PART) { return by_bn(M64{}, I4{}, K32{}, C128{}, W2{}, NO{}, NO{}, NO{}); } return -3;
    case 5: if constexpr (glds_part(5) == PART) { return by_bn(M256{}, I4{}, K32{}, C192{}, W4{}, NO{}, NO{}, NO{}); } return -3;
    case 6: if constexpr (glds_part(6) == PART) { return by_bn(M256{}, I3{}, K64{}, C128{}, W4{}, NO{}, NO{}, NO{}); } return -3;
    case 7: if constexpr (glds_part(7) == PART) { return by_bn(M256{}, I5{}, K32{}, C192{}, W4{}, NO{}, NO{}, NO{}); } return -3;
    case 8: if constexpr (glds_part(8) == PART) { return by_bn(M256{}, I3{}, K32{}, C128{}, W4{}, NO{}, NO{}, NO{}); } return -3;
    case 9: if constexpr (glds_part(9) == PART) { return by_bn(M128{}, I3{}, K32{}, C128{}, W2{}, ILV{}, NO{}, NO{}); } return -3;
    case 10: if constexpr (glds_part(10) == PART) { return by_bn(M128{}, I3{}, K32{}, C192{}, W2{}, ILV{}, NO{}, NO{}); } return -3;
    case 11: if constexpr (glds_part(11) == PART) { return by_bn(M128{}, I2{}, K64{}, C128{}, W2{}, ILV{}, NO{}, NO{}); } return -3;
    case 12: if constexpr (glds_part(12) == PART) { return by_bn(M256{}, I4{}, K32{}, C192{}, W4{}, ILV{}, NO{}, NO{}); } return -3;
    case 13: if constexpr (glds_part(13) == PART) { return by_bn(M256{}, I3{}, K32{}, C128{}, W4{}, ILV{}, NO{}, NO{}); } return -3;
    case 14: if constexpr (glds_part(14) == PART) { return by_bn(M256{}, I3{}, K32{}, C128{}, W4{}, NO{}, NO{}, WP4{}); } return -3;
    case 15: if constexpr (glds_part(15) == PART) { return by_bn(M256{}, I3{}, K32{}, C128{}, W4{}, ILV{}, NO{}, WP4{}); } return -3;
    case 16: if constexpr (glds_part(16) == PART) { return by_bn(M128{}, I3{}, K32{}, C128{}, W2{}, NO{}, NO{}, WP3{}); } return -3;
    case 17: if constexpr (glds_part(17) == PART) { return by_bn(M128{}, I3{}, K32{}, C128{}, W2{}, ILV{}, NO{}, WP3{}); } return -3;
    case 18: if constexpr (glds_part(18) == PART) { return by_bn(M128{}, I3{}, K32{}, C192{}, W2{}, NO{}, NO{}, WP2{}); } return -3;
    case 19: if constexpr (glds_part(19) == PART) { return by_bn(M64{}, I4{}, K32{}, C128{}, W2{}, NO{}, NO{}, WP3{}); } return -3;
    case 20: if constexpr (glds_part(20) == PART) { return by_bn(M64{}, I3{}, K32{}, C128{}, W2{}, NO{}, NO{}, WP4{}); } return -3;
    default: return -3;
  }
  }
}


}  // namespace glds
}  // namespace tony
