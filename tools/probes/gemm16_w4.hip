// One-wave-per-SIMD variant of the s16x3 input projection (round 5 probe, not shipped), included by
// tools/probes/gemm16_pp_probe.hip after gemm16.hip: bitwise equal to the persistent kernel, but
// 495 us against 415-433 us for gemm16_pp_kernel at Kp = 512 (profiles/r05/gemm16/).
namespace casr {
namespace {

// ---- one wave per SIMD (round 5 probe, not shipped: measured slower): four waves of 128 x 128 (4 x 4
// tiles of v_mfma_f32_32x32x16_f16), the 256 accumulation registers in AGPRs, each wave pipelining
// its own fragment reads: stage j + 1's 16 reads are issued among stage j's 48 MFMAs.  Against the two-group forms: a third fewer LDS reads per MFMA (a wave's A
// fragments feed 4 column tiles, its W fragments 4 row tiles) and no partner wave on the SIMD whose
// reads slow its MFMA sections.  The same ring as gemm16_pp_kernel (16-deep stages, four buffers,
// three in flight, scalar-base DMA), one barrier per stage:
//   top of iteration j: this wave's DMA of stage j + 1 retired (counted vmcnt), lgkmcnt(0), barrier
//   (stage j + 1 visible; every read of stage j - 1 done), DMA of stage j + 3 into stage j - 1's buffer,
//   then stage j's MFMAs with stage j + 1's reads (the next tile's stage 0 at a tile's last stage)
//   each issued right after the last use of the register it refills.  Epilogue per tile
// (after its last stage's MFMAs): 8 rounds of 16 rows x 128 columns per wave through a private 8 KB
// slab in the buffer of the tile's last stage, buffer stores (rows past M dropped: 64 per wave and
// tile).  Same per-element arithmetic as gemm16_persist_kernel: bitwise equal.
constexpr int W4_STORES = 64;  // buffer stores per wave and tile

template <int MAXY>
CASR_DEV void w4_vm_wait(int younger) {  // vmcnt(N): the largest of {63, 9, 8, 4, 0} not above younger
  if (younger >= 63) g16_vm_wait<63>();
  else if (younger >= 9) g16_vm_wait<9>();
  else if (younger >= 8) g16_vm_wait<8>();
  else if (younger >= 4) g16_vm_wait<4>();
  else g16_vm_wait<0>();
}

template <int DIAG = 0>
__global__ __launch_bounds__(256, 1) void gemm16_w4_kernel(const float* __restrict__ A16, const float* __restrict__ W16,
                                                           const float* __restrict__ bias, float* __restrict__ Cout,
                                                           int M, int N, int Kp, Order16 order, int total, int nk) {
  __shared__ __attribute__((aligned(16))) float lds[PP_LDS];
  asm volatile("; accumulators in AGPRs" ::: "a0");
  constexpr int NT = 4;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave >> 1, wn = wave & 1;
  const int r32 = lane & 31, hsel = lane >> 5;
  const int G = gridDim.x;
  const uint32_t lds_u32 = (uint32_t)(uintptr_t)(__attribute__((address_space(3))) float*)lds;
  float* const bias_lds = lds + PP_NBUF * PP_STAGE;
  auto next_tile = [&](int L, int& n, int& m) {
    while (L < total && !order.tile(L, n, m)) L += G;
    return L;
  };
  // DMA: this wave stages A rows [64 wave, +64) and W rows [64 wave, +64), four 16-row instructions each
  uint32_t vw[4];
  int coff[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int row = wave * 64 + i * 16 + (lane >> 2), c = (lane & 3) ^ ((row >> 2) & 3);
    coff[i] = (c >> 1) * 16 + (c & 1) * 4;
    vw[i] = (uint32_t)(row * Kp + coff[i]) * 4u;
  }
  auto a_offsets = [&](int m, uint32_t (&va)[4]) {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int row = wave * 64 + i * 16 + (lane >> 2);
      va[i] = (uint32_t)(min(row, M - 1 - m * G16_M) * Kp + coff[i]) * 4u;
    }
  };
  auto stage_dma = [&](int b, int n, int m, int s, int tpar, const uint32_t (&va)[4]) {
    if constexpr ((DIAG & 1) != 0) return;
    const int kb = (s >> 1) * 32 + (s & 1) * 8;
    const float* sa = A16 + (size_t)m * G16_M * Kp + kb;
    const float* sw = W16 + (size_t)n * G16_N * Kp + kb;
    const uint32_t l0 = lds_u32 + (uint32_t)(b * PP_STAGE + wave * 64 * PP_ROWF) * 4u;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      lds_dma16_s(va[i], sa, l0 + i * 16 * PP_ROWF * 4u);
      lds_dma16_s(vw[i], sw, l0 + (PP_OP + i * 16 * PP_ROWF) * 4u);
    }
    if (s == 0)
      lds_dma16_s((uint32_t)min(lane * 16, (N - n * G16_N - 4) * 4), bias + n * G16_N,
                  lds_u32 + (uint32_t)(PP_NBUF * PP_STAGE + tpar * G16_N) * 4u);
  };
  auto barrier = [] {
    __builtin_amdgcn_sched_barrier(0);
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_sched_barrier(0);
  };
  f32x16 acc[4][NT];
  const _Float16 two11 = (_Float16)2048.0f;
  // one register set of fragments: a stage's MFMAs run column tile by column tile, and each fragment
  // of the next stage is read into its register right after its last use (W of tile t after tile t's
  // 12 MFMAs; A of row tile tm after the last column tile's 3 MFMAs of it), so the reads fly under the
  // rest of the stage's MFMAs
  f16x8 wh[NT], wl[NT], ah[4], al[4];
  // per-lane float offsets of the fragments within a stage buffer (the swizzle (row >> 2) & 3 is the
  // same for every 32-row tile): tile t / tm adds 32 rows (immediate offsets of the ds_reads)
  const int sw = (r32 >> 2) & 3;
  const int off_wh = PP_OP + (wn * 128 + r32) * PP_ROWF + ((hsel ^ sw) << 2);
  const int off_wl = PP_OP + (wn * 128 + r32) * PP_ROWF + (((2 + hsel) ^ sw) << 2);
  const int off_ah = (wm * 128 + r32) * PP_ROWF + ((hsel ^ sw) << 2);
  const int off_al = (wm * 128 + r32) * PP_ROWF + (((2 + hsel) ^ sw) << 2);
  auto frag_w = [&](const float* buf, int t, f16x8& h, f16x8& l) {
    h = *reinterpret_cast<const f16x8*>(buf + off_wh + t * 32 * PP_ROWF);
    l = *reinterpret_cast<const f16x8*>(buf + off_wl + t * 32 * PP_ROWF);
  };
  auto frag_a = [&](const float* buf, int tm, f16x8& h, f16x8& l) {
    h = *reinterpret_cast<const f16x8*>(buf + off_ah + tm * 32 * PP_ROWF);
    l = *reinterpret_cast<const f16x8*>(buf + off_al + tm * 32 * PP_ROWF);
  };
  // stage j's MFMAs, the next stage's reads from buffer nb (after a tile's last stage with no next
  // tile: stale LDS, never used)
  auto mfma_stage = [&](const float* nb) {
#pragma unroll
    for (int t = 0; t < NT; ++t) {
      const f16x8 w1 = wh[t] * two11;
#pragma unroll
      for (int tm = 0; tm < 4; ++tm) {
        if constexpr ((DIAG & 2) == 0) {
          acc[tm][t] = __builtin_amdgcn_mfma_f32_32x32x16_f16(ah[tm], w1, acc[tm][t], 0, 0, 0);
          acc[tm][t] = __builtin_amdgcn_mfma_f32_32x32x16_f16(ah[tm], wl[t], acc[tm][t], 0, 0, 0);
          acc[tm][t] = __builtin_amdgcn_mfma_f32_32x32x16_f16(al[tm], wh[t], acc[tm][t], 0, 0, 0);
        } else if (ah[tm][0] == (_Float16)1234.f && w1[0] == (_Float16)4321.f) {
          acc[tm][t][0] += 1.f;
        }
        if (t == NT - 1) frag_a(nb, tm, ah[tm], al[tm]);
      }
      frag_w(nb, t, wh[t], wl[t]);
    }
  };

  int n, m;
  int L = next_tile(blockIdx.x, n, m);
  if (L >= total) return;
  int n2 = n, m2 = m;
  int L2 = next_tile(L + G, n2, m2);
  int gb = 0, tpar = 0;
  uint32_t va[4], va2[4];
  a_offsets(m, va);
  a_offsets(m2, va2);
  for (int s = 0; s < 3; ++s) stage_dma(s, n, m, s, 0, va);
  w4_vm_wait<63>((DIAG & 1) ? 0 : 16);  // stage 0 and its bias landed: younger = stages 1, 2
  barrier();
#pragma unroll
  for (int t = 0; t < NT; ++t) frag_w(lds, t, wh[t], wl[t]);
#pragma unroll
  for (int tm = 0; tm < 4; ++tm) frag_a(lds, tm, ah[tm], al[tm]);
  bool after_epi = false;
  while (true) {
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int t = 0; t < NT; ++t)
#pragma unroll
        for (int e = 0; e < 16; ++e) acc[i][t][e] = 0.f;
    auto ex = [&](int s) { return s < nk || L2 < total; };
    auto ops = [&](int s) { return ex(s) ? 8 + (s == nk ? 1 : 0) : 0; };
    for (int j = 0; j < nk; ++j) {
      // VMEM operations issued after this wave's DMA of stage j + 1: stage j + 2's, and the previous
      // tile's epilogue stores while stages 1 and 2 of a tile wait (capped: vmcnt counts to 63)
      const int younger = (DIAG & 1) ? 0 : ops(j + 2) + (after_epi && j < 2 ? W4_STORES : 0);
      if (j + 1 < nk || L2 < total) w4_vm_wait<63>(younger);
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      barrier();
      const int s3 = j + 3;
      if (s3 < nk) stage_dma((gb + s3) & 3, n, m, s3, tpar, va);
      else if (L2 < total) stage_dma((gb + s3) & 3, n2, m2, s3 - nk, tpar ^ 1, va2);
      int nb = ((gb + j + 1) & 3) * PP_STAGE;
      nb = __builtin_amdgcn_readfirstlane(nb);
      asm volatile("" : "+s"(nb));  // computed here, not hoisted per buffer out of the loop
      mfma_stage(lds + nb);
    }
    // ---- epilogue: per wave, 8 rounds of 16 rows x 128 columns through a private 8 KB slab in the
    // buffer of the tile's last stage (free: every wave's reads of it retired before the last barrier)
    {
      float* slab = lds + ((gb + nk - 1) & 3) * PP_STAGE + wave * 16 * 128;
      const int c4 = lane & 31, rq = lane >> 5;
      const float4 b4 = *reinterpret_cast<const float4*>(bias_lds + tpar * G16_N + wn * 128 + c4 * 4);
      const int m0 = m * G16_M;
      const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(
          Cout + (size_t)m0 * N, 0, (int)((size_t)min(G16_M, M - m0) * N * 4), 0x00020000);
      int cbase = n * G16_N + wn * 128 + c4 * 4;
      int lrow = wm * 128 + rq;  // (lane-dependent offsets opaque here: not hoisted out of the tile loop)
      asm volatile("" : "+v"(cbase), "+v"(lrow));
#pragma unroll
      for (int tm = 0; tm < 4; ++tm)
#pragma unroll
        for (int hh = 0; hh < 2; ++hh) {
#pragma unroll
          for (int t = 0; t < NT; ++t)
#pragma unroll
            for (int e = 8 * hh; e < 8 * hh + 8; ++e)
              slab[((e & 3) + 8 * ((e >> 2) & 1) + 4 * hsel) * 128 + t * 32 + r32] = acc[tm][t][e] * S16_LO_INV;
          asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
#pragma unroll
          for (int i = 0; i < 8; ++i) {
            const int row = rq + 2 * i;
            const float4 v = *reinterpret_cast<const float4*>(slab + row * 128 + c4 * 4);
            const int lr = lrow + tm * 32 + 16 * hh + 2 * i;
            const float4 o = make_float4(v.x + b4.x, v.y + b4.y, v.z + b4.z, v.w + b4.w);
            if (!(DIAG & 4))
              __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, o), rs, (lr * N + cbase) * 4, 0, 0);
            else if (v.x == 12345.f)
              Cout[0] = o.x;
          }
          asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        }
    }
    if (L2 >= total) break;
    gb = (gb + nk) & 3;
    L = L2;
    n = n2;
    m = m2;
    tpar ^= 1;
    after_epi = !(DIAG & 4);
    L2 = next_tile(L + G, n2, m2);
    va[0] = va2[0], va[1] = va2[1], va[2] = va2[2], va[3] = va2[3];
    a_offsets(m2, va2);
  }
}

}  // namespace
}  // namespace casr
