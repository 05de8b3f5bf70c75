// The layer body of conv_stack_f8_kernel (conv_stack_f8.hip), included textually in the
// kernel's layer loops, twice by every variant but C = 256 backward-data: the non-last layers'
// loop (lean epilogue, compile-time last = false) and the last layer (general epilogue) then
// get their own register allocation instead of one for the union of both in one rolled loop
// (C = 128 barrier forward 256 VGPRs + 8 spills -> 238 + 0, staggered forward 256 + 8 -> 242 +
// 0: 10 layers 153.8 -> 144.2 us).  Why an include: the same text wrapped in an always_inline
// lambda allocated differently — the staggered variants spilled 5-23 VGPRs inside the K loop.  Expects the
// kernel's locals in scope and `l` (layer index) and `last` (last layer) defined.
// Not a header: no include guard, included only inside conv_stack_f8_kernel.
  if constexpr (C == 128) make_pk();
  if constexpr (STAG) img_rd = (l & 1) * IMG2;
  const F8Layer L = a.L[l];
  const char* A_next = l + 1 < a.nl ? a.L[l + 1].A8 : L.A8;
  const F8Layer Lprev = a.L[l > 0 ? l - 1 : 0];
  const bool co_on = l > 0;
  char* co_yb = (MODE & 16) ? nullptr : Lprev.Y + (size_t)b * FF * C * 2;
  uint8_t* co_y8b = Lprev.Y8 ? Lprev.Y8 + (size_t)b * FP8P * C : nullptr;
  const float s_x = *L.s_in;
  const float deq = s_x * *L.s_w;
  const float inv_y = 1.f / *L.s_out;
  float vmax = 0.f;
  uint4 co_v;

  for (int hp = 0; hp < NC; ++hp) {     // output pass: channels 128 hp .. 128 hp + 127
    const char* Ap = L.A8 + (size_t)hp * G::STEPS * STEP_BYTES;
    // the A fragments to prefetch after this pass's last step: the next pass / layer
    const char* A_after = hp + 1 < NC ? Ap + G::STEPS * STEP_BYTES : A_next;
    f32x4 acc[MF][NF];
#pragma unroll
    for (int i = 0; i < MF; ++i)
#pragma unroll
      for (int j = 0; j < NF; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

    // (structure of conv_stack2's K loop: rolled, sched_barrier-pinned plain loads, each
    // half of the A fragments re-loaded right after its MFMAs, copy-out store last)
    auto kstep = [&](const int st, const int cs, const bool co) {
      const char* An = st + 1 < G::STEPS ? Ap + (st + 1) * STEP_BYTES : A_after;
      i32x8 bfr[NF];
      if constexpr ((MODE & 128) != 0) {
        // (ablation: no B reads — opaque register operands)
#pragma unroll
        for (int j = 0; j < NF; ++j) {
          int z = (int)pk[j];
          asm volatile("" : "+v"(z));
          bfr[j] = i32x8{z, z, z, z, z, z, z, z};
        }
      } else {
        read_B(st, bfr);
      }
      mma(Ak, 0, bfr, acc);
      __builtin_amdgcn_sched_barrier(0);
      if constexpr (!(MODE & 2)) load_A(An, 0, Ak);
      if (co) co_v = co_read(cs);
      __builtin_amdgcn_sched_barrier(0);
      mma(Ak, 2, bfr, acc);
      __builtin_amdgcn_sched_barrier(0);
      if constexpr (!(MODE & 2)) load_A(An, 2, Ak);
      if (co) co_store(cs, co_v, co_yb, co_y8b, Lprev.mask, s_x);
      __builtin_amdgcn_sched_barrier(0);
    };
    // the copy-out steps (the first CO_STEPS of pass 0) and the rest as separate loops
    // (no per-step branch; the step index laundered so the compiler does not precompute
    // every step's copy-out addresses)
    if constexpr (C == 128) {
      // half-major K-steps (read_B): 0..3 channels 0..63, 4 both halves, 5..8 channels
      // 64..127.  Staggered schedule (STAG): no workgroup barrier between the layers of
      // the run, and a double-buffered image.  A wave reads image half c of a layer once
      // co-half c has written it (W_c: 4 waves per layer) — half 0 from step 0, half 1 from
      // step 4; a group writes its output into the other image as soon as its K loop ends
      // (that image was layer l - 1's input: every wave is past those reads, since each
      // group waited for the other's layer l - 1 output inside layer l).  The co-halves
      // drift apart (the older waves win issue arbitration: co-half 0 finishes its K loop
      // ~30% earlier), so co-half 0's epilogue runs beside co-half 1's last K-steps and
      // co-half 1's beside co-half 0's first four, instead of idling the MFMA pipes between
      // two barriers.  The copy-out (steps 0..5) of each half is done by its own co-half
      // (own writes: W_wm).
      stamp(l, 0);
      if constexpr (STAG) {
        grp_wait(cnt + 2, 4u * (unsigned)l);                        // W0
        if (wm == 1) grp_wait(cnt + 3, 4u * (unsigned)l);           // W1 (own copy-out)
      }
      stamp(l, 1);
      int st = 0;
      if (!(MODE & 4) && co_on) {
#pragma unroll 1
        for (; st < G::CO_STEPS; ++st) {
          int tt = st;
          asm volatile("" : "+s"(tt));
          if constexpr (STAG) grp_wait_at(cnt + 3, 4u * (unsigned)l, tt, 4);   // W1
          kstep(tt, tt, true);
        }
      }
#pragma unroll 1
      for (; st < G::STEPS; ++st) {
        int tt = st;
        asm volatile("" : "+s"(tt));
        if constexpr (STAG) grp_wait_at(cnt + 3, 4u * (unsigned)l, tt, 4);     // W1
        kstep(tt, 0, false);
      }
      stamp(l, 2);
    } else {
      int st = 0;
      if (!(MODE & 4) && co_on && hp == 0) {
#pragma unroll 1
        for (; st < G::CO_STEPS; ++st) {
          int tt = st;
          asm volatile("" : "+s"(tt));
          kstep(tt, tt, true);
        }
      }
#pragma unroll 1
      for (; st < G::STEPS; ++st) kstep(st, 0, false);
    }

    // ---- pass epilogue ----
    if constexpr ((MODE & 64) != 0) {
      // (ablation: no epilogue — the accumulators only feed the amax)
#pragma unroll
      for (int i = 0; i < MF; ++i)
#pragma unroll
        for (int j = 0; j < NF; ++j) vmax = fmaxf(vmax, acc[i][j][0]);
      if (C == 128 || hp == NC - 1) lds_barrier();
      continue;
    }
    // an opaque zero added to the epilogue's addresses: otherwise the compiler hoists all
    // per-fragment table / LDS addresses out of the layer loop and spills them
    int z0 = 0;
    asm volatile("" : "+v"(z0));
    // EPI_FWD: bias table pieces; EPI_DGRAD: the 64 ReLU bits (of the layer below) of this
    // wave's channels per pixel fragment
    uint2 eb[NF][EPI == EPI_FWD ? MF : 1];
    uint2 em[NF];
#pragma unroll
    for (int j = 0; j < NF; ++j) {
      if constexpr (EPI == EPI_FWD) {
        const uint2* pf = (const uint2*)L.pbias + hp * (24 * 2 * 4 * 64) +
                          ((wn * NF + j) * 2 + wm) * 4 * 64 + lane + z0;
#pragma unroll
        for (int i = 0; i < MF; ++i) eb[j][i] = pf[i * 64];
      } else {
        const int p = min(wn * NF * 16 + j * 16 + lr, NPTS - 1);
        em[j] = *(const uint2*)(L.mask + ((size_t)b * NPTS + p) * (C / 8) + 16 * hp + 8 * wm + z0);
      }
    }
    // C = 128 and the last pass of C = 256: every wave is past its last read of the
    // image before it is overwritten (pass 0 of C = 256 only writes the park area)
    const bool to_image = !last && hp == NC - 1;
    // (STAG, non-last layers: no wait — the output goes into the other image)
    if (!(STAG && !last) && (C == 128 || hp == NC - 1)) lds_barrier();
    stamp(l, 3);
    char* sIe = smem + SCRATCH + z0;
    // (the lean epilogue's output image: STAG writes the other one)
    const int img_wr = STAG ? IMG2 - img_rd : 0;
    if (BF16_LAST_IMAGE && last) {
      // the bf16 two-image layout needs zero border rows (and rows 441..447, which the
      // head's weight-gradient pass reads against zero dz): the region held e4m3 data
      for (int u = tid; u < 87 * 8 * 2; u += NT) {
        const int img = u / (87 * 8), k = (u >> 3) % 87, q = u & 7;
        const int row = k < 21 ? k : k < 42 ? 420 + (k - 21) : k < 61 ? (k - 41) * 21
                        : k < 80 ? (k - 60) * 21 + 20 : 441 + (k - 80);
        *(uint4*)(sIe + img * H_BYTES + row * 128 + q * 16) = uint4{0, 0, 0, 0};
      }
    }
    // stochastic-rounding key of this lane's first element (fragment (0, 0)) in this pass
    uint32_t sr_lane = 0;
    if constexpr (EPI == EPI_DGRAD && (MODE & 32) != 0)
      sr_lane = sr_seed + (uint32_t)(l + 1) * 0x85EBCA6Bu +
                (uint32_t)((b * NPTS + wn * NF * 16 + lr) * C + 128 * hp + wm * 64 + lq * 4);
    if (!last && (C == 128 || EPI == EPI_DGRAD)) {
      // (C = 256 forward: the general loop — its lean form spilled 20 VGPRs and measured
      // +1.5%; the backward-data one -12%, profiles/r5_stack_f8_stag.txt)
      // Lean epilogue (non-last layers): straight-line — no per-fragment branch (C = 128:
      // the pixels past the board store to the dump rows; C = 256, whose LDS has no room
      // for them: the store of fragment columns 4 and 5 only, where such pixels occur, is
      // lane-masked; a select keeps them out of the |y| max), one XOR per fragment for its
      // LDS address, and per value: forward fma + ReLU max + scale + clamp; backward-data
      // mask AND (v_bfe_i32 gives the lane mask) + scale + clamp, the |dz| max taken before
      // the dequantization.  Same results as the general loop below (the output scale is a
      // power of two).
      const float s1 = EPI == EPI_FWD ? inv_y : deq * inv_y;
      float m_all = 0.f;
#pragma unroll
      for (int j = 0; j < NF; ++j) {
        uint32_t pkj = pk[j];
        asm volatile("" : "+v"(pkj));
        // image: row + byte lq*4 + slot (8hp + 4wm ^ sig) << 4, fragment i's slot is
        // (8hp + 4wm + i) ^ sig; C = 256 pass 0 parks pixel p's row (piece (cl / 16) ^
        // (p & 7), general loop below) — the same XOR by i << 4 either way
        const int pj = wn * NF * 16 + j * 16 + lr;
        uint32_t a_j = ((pkj & 0xFFFFFu) + (uint32_t)(lq * 4)) |
                       ((uint32_t)((8 * hp + 4 * wm) ^ sig_of<C>((int)(pkj >> 20))) << 4);
        if (C == 256 && !to_image) {
          const int pr = pj < G::PARK1 ? pj * 128 : SCRATCH + G::IMG + (pj - G::PARK1) * 128;
          a_j = (uint32_t)(pr - SCRATCH) + (uint32_t)((wm * 64 + lq * 4) ^ ((lane & 7) << 4));
        }
        uint32_t wx = 0, wy = 0;
        if constexpr (EPI == EPI_DGRAD) {
          wx = em[j].x >> (lq * 4);
          wy = em[j].y >> (lq * 4);
        }
        float mj = 0.f;
#pragma unroll
        for (int i = 0; i < MF; ++i) {
          const f32x4 v = acc[i][j];
          float x[4];
          if constexpr (EPI == EPI_FWD) {
            const uint2 u = eb[j][i];
            x[0] = fmaxf(fmaf(v[0], deq, __uint_as_float(u.x << 16)), 0.f);
            x[1] = fmaxf(fmaf(v[1], deq, __uint_as_float(u.x & 0xFFFF0000u)), 0.f);
            x[2] = fmaxf(fmaf(v[2], deq, __uint_as_float(u.y << 16)), 0.f);
            x[3] = fmaxf(fmaf(v[3], deq, __uint_as_float(u.y & 0xFFFF0000u)), 0.f);
            mj = fmaxf(mj, fmaxf(fmaxf(x[0], x[1]), fmaxf(x[2], x[3])));
#pragma unroll
            for (int r = 0; r < 4; ++r) x[r] = fminf(x[r] * s1, QMAX);
          } else {
            const uint32_t w = (i < 2 ? wx : wy) >> ((i & 1) * 16);
#pragma unroll
            for (int r = 0; r < 4; ++r)
              x[r] = __uint_as_float(__float_as_uint(v[r]) &
                                     (uint32_t)__builtin_amdgcn_sbfe((int)w, r, 1));
            mj = fmaxf(mj, fmaxf(fmaxf(fabsf(x[0]), fabsf(x[1])),
                                 fmaxf(fabsf(x[2]), fabsf(x[3]))));
#pragma unroll
            for (int r = 0; r < 4; ++r) x[r] = __builtin_amdgcn_fmed3f(x[r] * s1, -QMAX, QMAX);
          }
          const uint32_t key = sr_lane + (uint32_t)(j * 16 * C + i * 16);
          const uint32_t q8 = pack8x4q<EPI, MODE>(x[0], x[1], x[2], x[3], key);
          // (C = 256: columns 0..3 hold board pixels only, wn * 96 + 63 < 361)
          if (C == 128 || j < 4 || pj < NPTS)
            *(LDS_AS uint32_t*)((LDS_AS char*)sIe + img_wr + (a_j ^ (uint32_t)(i << 4))) = q8;
        }
        m_all = fmaxf(m_all, pj < NPTS ? mj : 0.f);
        __builtin_amdgcn_sched_barrier(0);   // (one fragment column at a time)
      }
      vmax = fmaxf(vmax, EPI == EPI_FWD ? m_all : m_all * deq);
    } else
#pragma unroll
    for (int j = 0; j < NF; ++j) {
      const int p = wn * NF * 16 + j * 16 + lr;
      // offsets from an opaque copy of pk[j]: visible, the compiler hoists every
      // (fragment, slot) offset out of the layer loop and spills them (conv_stack2.hip)
      uint32_t pkj = pk[j];
      asm volatile("" : "+v"(pkj));
      const int f = (int)(pkj & 0xFFFFFu) / ROWB;
      const int sig = sig_of<C>((int)(pkj >> 20));
#pragma unroll
      for (int i = 0; i < MF; ++i) {
        f32x4 v = acc[i][j];
        if constexpr (EPI == EPI_FWD) {
          const uint2 u = eb[j][i];
          v[0] = fmaxf(v[0] * deq + __uint_as_float(u.x << 16), 0.f);
          v[1] = fmaxf(v[1] * deq + __uint_as_float(u.x & 0xFFFF0000u), 0.f);
          v[2] = fmaxf(v[2] * deq + __uint_as_float(u.y << 16), 0.f);
          v[3] = fmaxf(v[3] * deq + __uint_as_float(u.y & 0xFFFF0000u), 0.f);
        } else {
          const int cw = i * 16 + lq * 4;                // channel within the wave's 64
          const uint32_t word = (cw < 32) ? em[j].x : em[j].y;
          const uint32_t bits = word >> ((cw & 31) >> 3 << 3) >> (cw & 4);
#pragma unroll
          for (int r = 0; r < 4; ++r) v[r] = ((bits >> r) & 1u) ? v[r] * deq : 0.f;
        }
        if (p >= NPTS) continue;
        const int cl = wm * 64 + i * 16 + lq * 4;      // channel within the pass (0..127)
        if (!last) {
          vmax = fmaxf(vmax, fmaxf(fmaxf(fabsf(v[0]), fabsf(v[1])), fmaxf(fabsf(v[2]), fabsf(v[3]))));
          auto qz = [&](float x) { return fmaxf(fminf(x * inv_y, QMAX), -QMAX); };
          // (key: layer l + 1's seed + the element index (b, p, co); the prologue is layer 0)
          const uint32_t key = sr_lane + (uint32_t)(j * 16 * C + i * 16);
          const uint32_t q8 = pack8x4q<EPI, MODE>(qz(v[0]), qz(v[1]), qz(v[2]), qz(v[3]), key);
          if (to_image) {
            // channel co = 128 hp + cl: slot co / 16 (XOR sig), byte co % 16
            const int co = 128 * hp + cl;
            *(uint32_t*)(sIe + f * ROWB + (((co >> 4) ^ sig) * 16) + (co & 15)) = q8;
          } else {
            // C = 256 pass 0: park (pixel-major 128-B rows) in the LDS around the image.
            // 16-B piece cl / 16 of pixel p sits at piece (cl / 16) ^ (p & 7): unswizzled,
            // the 16 pixels of a store (rows 128 B apart) hit one bank — a 16-way conflict
            // on every parked store (~15M conflict cycles per 12x256 launch); now 2-way (32
            // lanes over 8 pieces x 2 words): 18.0M / 16.4M -> 6.4M / 4.8M conflict cycles
            // per launch (profiles/r4_s1_early_update_park_ab.txt).  (p & 7 == lane & 7: a fragment's
            // 16 pixels start at a multiple of 16)
            char* pr = p < G::PARK1 ? smem + p * 128
                                    : smem + SCRATCH + G::IMG + (p - G::PARK1) * 128;
            *(uint32_t*)(pr + z0 + (cl ^ ((lane & 7) << 4))) = q8;
          }
        } else if constexpr (BF16_LAST_IMAGE) {
          // bf16 two-image layout (conv_stack2 / head_body.h) for the fused head
          const int cw = i * 16 + lq * 4;
          uint2 o;
          o.x = pack_bf16x2(v[0], v[1]);
          o.y = pack_bf16x2(v[2], v[3]);
          *(uint2*)(sIe + wm * H_BYTES + f * 128 + (((cw >> 3) ^ fsig8(f)) * 16) + (cw & 4) * 2) = o;
        } else {
          // last layer (C = 256 forward, any dgrad): bf16 straight to the output frame
          // (+ the forward's ReLU bits)
          const int co = 128 * hp + cl;
          uint2 o;
          o.x = pack_bf16x2(v[0], v[1]);
          o.y = pack_bf16x2(v[2], v[3]);
          *(uint2*)(L.Y + ((size_t)(b * FF + f) * C + co) * 2 + z0) = o;
          if constexpr (EPI == EPI_FWD) {
          const uint32_t nib = (v[0] > 0.f ? 1u : 0u) | (v[1] > 0.f ? 2u : 0u) |
                               (v[2] > 0.f ? 4u : 0u) | (v[3] > 0.f ? 8u : 0u);
          // 4 bits of one mask byte: the lane pair (lq even, odd) shares the byte
          const uint32_t other = __shfl_xor(nib, 16, 64);
          if ((lq & 1) == 0)
            L.mask[((size_t)b * NPTS + p) * (C / 8) + (co >> 3) + z0] = (uint8_t)(nib | (other << 4));
          }
        }
      }
    }
    if (C == 256 && to_image) {
      // pass 0's parked half into the image (every wave is past the barrier above, and
      // every parked write precedes it in this wave... all waves: barrier first)
      lds_barrier();
      for (int u = tid; u < NPTS * 8; u += NT) {     // 16-B pieces of channels 0..127
        const int p = u >> 3, q = u & 7;
        const char* pr = p < G::PARK1 ? smem + p * 128
                                      : smem + SCRATCH + G::IMG + (p - G::PARK1) * 128;
        const uint4 v = *(const uint4*)(pr + z0 + ((q ^ (p & 7)) * 16));
        const int h = p / BOARD, w = p - (p / BOARD) * BOARD;
        const int f = (h + 1) * F + (w + 1);
        *(uint4*)(sIe + f * ROWB + ((q ^ fsig<C>(f)) * 16)) = v;
      }
    }
  }
  if (STAG && !last) {
    grp_signal(cnt + 2 + wm);                                    // W_wm
    const float m = wave_max(vmax);
    if (lane == 0)
      __hip_atomic_fetch_max(s_lmax + l, __float_as_uint(m), __ATOMIC_RELAXED,
                             __HIP_MEMORY_SCOPE_WORKGROUP);
    stamp(l, 4);
  } else {
    if (!last) wg_amax(vmax, L.amax_out, s_amax + 8 * (l & 1));  // (barrier inside)
    stamp(l, 4);
    lds_barrier();  // the next layer's input is complete
    stamp(l, 5);
  }
