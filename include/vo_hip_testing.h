/* Test-only entry points of libvo_hip.so.  Not part of the product surface (vo_hip.h):
 * nothing in src/main.py's path calls them; the parity tests (tests/) do. */
#ifndef VO_HIP_TESTING_H
#define VO_HIP_TESTING_H

#include "vo_hip.h"

#ifdef __cplusplus
extern "C" {
#endif

/* Test stand-in for vo_comm_init: nranks contexts of ONE process (any devices, one host
 * thread each) join the in-process group named by the 128-byte id; all-reduces go
 * through host memory in rank order.  Exercises the sharded path where RCCL cannot
 * (RCCL refuses two ranks on one device).  Not a transport for production. */
int vo_comm_init_loopback(vo_ctx* ctx, int nranks, int rank, const char id[128]);

/* Test/tool switch: on != 0 keeps the BA's slab reduction (K2) a launch of its own on this
 * context, as on more than one rank (where the all-reduce sits between K2 and the solve);
 * by default one rank runs K2 inside the banded solve's launch.  Results are identical
 * either way (same sums).  tools/shard_projection.py times the multi-rank layout with it. */
int vo_ba_split_reduce(vo_ctx* ctx, int on);

/* Test switch: n > 0 launches every fused slab-reduction + solve of this context with n fewer
 * reducer workgroups than its solver waits for, so the solver's bounded wait times out (about
 * a quarter of a second per launch).  vo_ba_run / vo_ba_gn_step then return VO_ERR_HIP naming
 * the timeout, with the state left at the failed iteration's linearisation point, as for a
 * failed factorisation.  n = 0 restores normal launches. */
int vo_ba_testing_drop_reducers(vo_ctx* ctx, int n);

/* Test switch: the K1 variant this context's later vo_ba_setup calls plan.  0: the default
 * (the one-wave K1 with six chunks per segment while they fit one round of workgroups, else
 * three); -1: the four-wave K1 (segments of several chunks of one first-camera group, one
 * 256-lane workgroup walking them); n = 1 .. 6: the one-wave K1 with n chunks of one first-camera
 * group per segment (one wave per chunk, the segment's waves in one workgroup summing their slot
 * blocks in chunk order: one slab row per segment slot).  Same arithmetic, different summation
 * order: results agree to rounding, all within the oracle tolerance.  Keeps every K1 variant
 * covered by the GPU tests; takes effect at the next setup. */
int vo_ba_testing_k1(vo_ctx* ctx, int variant);

/* Test switch: on != 0 keeps this context's later vo_ba_setup calls off the banded solver's
 * split layout (two workgroups, one per side), so a window too large for one workgroup's LDS
 * takes the ring layout (factor records in global memory) as before round 6.  Same arithmetic:
 * the GPU tests compare the two layouts bitwise.  Takes effect at the next setup. */
int vo_ba_testing_no_split(vo_ctx* ctx, int on);

/* Host only: the digest (as vo_ba_plan_digest) of the plan of `cur` packed for seg_obs
 * observations per segment (seg_obs 1: the one-wave K1's plan of seg_chunks chunks per
 * segment), built from scratch when prev is NULL, else after a from-scratch plan of `prev`
 * (same packing) as vo_ba_setup builds it on a window slide: taking over prev's unchanged
 * first-camera groups.  *reused_chunks (may be NULL): chunks taken over. */
int vo_ba_testing_plan_slide(const vo_ba_problem* prev, const vo_ba_problem* cur, int seg_obs, int seg_chunks,
                             uint64_t* digest, int64_t* reused_chunks);

/* Test/tool switch for this context's PnP calls (vo_pnp_ransac*): h1 > 0 solves and scores
 * the first h1 hypotheses of every frame, replays the serial RANSAC loop over them and solves
 * the rest only for the frames whose loop goes on; h1 = 0 (default) does that for batches of
 * more hypotheses than one wave per SIMD holds, h1 sized to that; h1 = -1 solves all at once.
 * Results are identical in every mode. */
int vo_pnp_testing_split(vo_ctx* ctx, int h1);

/* Synchronises the context stream and reports the last PnP call: *h1 hypotheses solved for
 * every frame, *tail_frames frames whose hypotheses [h1, iterations) were solved too. */
int vo_pnp_testing_last_split(vo_ctx* ctx, int* h1, int* tail_frames);

/* Test switch: the EPnP hypothesis kernel of the context's PnP calls.  0: the default (lane
 * groups while the hypotheses fit one wave per SIMD, else one lane per hypothesis); 1: lane groups
 * always; -1: one lane per hypothesis always.  Both kernels compute the same bits (the groups'
 * Jacobi steps are the serial sweep's rotations in the same order per row), which the GPU tests
 * check on one batch through both. */
int vo_pnp_testing_group(vo_ctx* ctx, int mode);

#ifdef __cplusplus
}
#endif
#endif /* VO_HIP_TESTING_H */
