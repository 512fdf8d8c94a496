// variants.hpp -- the compile-time tuning switches of the hot kernels, in one place.
//
// Each default below is the measured winner on MI355X (DESIGN.md section 4 has the A/B numbers). A
// variant library is built with other values by tools/build_variant.sh <name> "-DNAME=value ..." into
// randblas_amd/_var/<name>.so and timed with RBH_LIB_PATH pointing at it (tools/variants.sh); the
// product library always uses these defaults. Settings measured as losing were removed from the
// source, not kept as switches.
#pragma once

// ---- skge_dense.hip: the streamed GEMM (skge_stream_kernel) ---------------------------------
// memory-operand prefetch depth, in part-blocks ahead of their use: f64 7 (64 x 512 tiles: C2 7.97-7.98
// ms against 7.99-8.02 with 3; 32 x 1024 tiles: C2 7.66-7.68 against 7.70-7.71 with 3, C5 3.91 against
// 4.02-4.08; with rounds of 8, NS 15.27-15.30 against 15.43-15.46 with 3), f32 3 (C4 4.08-4.11 against
// 4.18-4.20 with 1), the one-triangle forms 3 since the rounds of 8 (C5p kernel 4.084-4.089 ms against
// 4.158-4.177 with 7 and 4.36-4.38 with 1; profiles/r06/ab_pf_tri.jsonl)
#ifndef RBH_PF64
#define RBH_PF64 7
#endif
#ifndef RBH_PF32
#define RBH_PF32 3
#endif
#ifndef RBH_PF_TRI
#define RBH_PF_TRI 3
#endif
// prefetch depth of the 32-row transposed-operand forms (TRI 5; their part-blocks are four 8-B
// loads): f64 32 x 1024 PF 7 7.74-7.77 ms against 7.80-7.82 with 3 at d = 1024, m = n = 16384, same
// box, two alternations (with rounds of 8: 7.64-7.67 against 7.72-7.75, profiles/r06/ab_pf_stream.jsonl)
#ifndef RBH_PF_TRI32
#define RBH_PF_TRI32 7
#endif
// one-triangle symmetric operands (sketch_symmetric_triangle, packed A): 1 = the streamed kernel
// on 64 x 512 tiles (C5p 4.25-4.26 ms against 4.59-4.61 with 0), 0 = skge_wide_kernel's LDS transpose
// of the mirrored tiles (the materialised-window option always takes it). (Round 5's RBH_TRI_WIDE,
// the one-triangle operand on the full-storage call's 32 x 1024 tiles, measured 5.5 ms against 4.26
// and spilled ring registers: removed, see launch_stream.)
#ifndef RBH_TRI_STREAMED
#define RBH_TRI_STREAMED 1
#endif

// steps per round of the streamed f64 kernel (one barrier per round; the next round's generated tiles
// are drawn during it; the LDS ring holds two rounds). 32-row tiles 8 (NS 15.32-15.34 ms against
// 15.36-15.41, NS RowMajor 15.36-15.38 against 15.47-15.51, C2 7.672-7.677 against 7.690-7.702; 16:
// a kilobyte a lane of spills), one-triangle operands 8 (C5p 4.161-4.164 ms against 4.223-4.227);
// the 64 x 512 tiles of a full-storage operand keep 4: beside sketch_symmetric's check a 128-KiB
// ring leaves it no LDS (C5 step 4.56-4.78 ms against 4.17-4.20). Same box, alternating
// (profiles/r06/ab_stream_r8.jsonl, ab_stream_r8_bench.jsonl).
#ifndef RBH_STREAM_R32
#define RBH_STREAM_R32 8
#endif
#ifndef RBH_STREAM_RTRI
#define RBH_STREAM_RTRI 8
#endif

// ---- saso.hip: the LDS-DMA SASO apply (saso_dma_kernel) --------------------------------------
// log2 of the chunk depth (contracted indices per panel): 7 (64-deep chunks: 0.70-0.84 ms on C3)
#ifndef SD_KCS_DEF
#define SD_KCS_DEF 7
#endif
// panel buffers in the LDS ring, and panels in flight ahead of the walked one
#ifndef SD_NB_DEF
#define SD_NB_DEF 2
#endif
#ifndef SD_PD_DEF
#define SD_PD_DEF 1
#endif
// pad each panel column by 8 B instead of XOR-swizzling its 16-B slots (conflict-free b64 reads)
#ifndef SD_PAD8_DEF
#define SD_PAD8_DEF 1
#endif
// waves that issue the panel copies (4: C3 0.57 ms; 8 0.58, 2 0.81, 16 0.61)
#ifndef SD_CW_DEF
#define SD_CW_DEF 4
#endif
