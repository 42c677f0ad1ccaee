/*
 * tray_debug.h — test and A/B hooks of libtray_amd.so. NOT part of the stable
 * C-ABI in tray.h: names and meanings may change with any build, and a
 * production caller (e.g. the cgo shim of INTEGRATION.md) never calls them.
 *
 * The library never reads the process environment: a stray TRAY_* variable in a
 * host process cannot change what it renders. The knobs below are process-wide
 * and apply to renders started after the call; unset knobs keep the product
 * behaviour. Each knob overrides one decision the library otherwise makes
 * itself; the frames they produce stay bit-identical to the defaults unless
 * noted (tests/test_gpu_*.py check exactly that).
 *
 *   "acc_slots"           on-chip chunk accumulators per wave (0 = off: chunk
 *                         sums through the per-sample buffer; same bits)
 *   "band_samples"        samples per launch band (< 2^30; < 2^31 with on-chip
 *                         chunk sums): splits a render into
 *                         more launches (same bits)
 *   "bvh_leaf"            BVH leaf size 1, 2 or 4 at tray_scene_upload (same bits)
 *   "bvh_lds_mode"        force LDS layout 0 / 1 / 2 when it fits (same bits)
 *   "stack_lds_slots"     cap the traversal stack's LDS slots (overflow path; same bits)
 *   "node_deep"           0 / 1: the 5- or 6-node-step kernel instance (same bits)
 *   "primary_candidates"  0: camera rays traverse the BVH instead of their
 *                         pixel's candidate list (same bits)
 *   "resolve_staged"      0: the plain per-pixel resolve instead of the LDS-staged
 *                         one for the per-sample buffer (the ordered FP64 sum, and
 *                         the fixed-point sums without on-chip slots) (same bits)
 *   "wave_chunks"         chunks a wave reserves per work-queue take (1..64), for
 *                         the whole launch (default: the build's size, single
 *                         chunks near the end of the queue) (same bits)
 *   "scene_contexts"      launch contexts per scene (default 4): renders of one
 *                         scene beyond this many in flight wait for the least
 *                         recently used one; 1 serialises them (same bits)
 *   "grid_reserve"        workgroup slots the persistent render grid leaves
 *                         free, out of the workgroups the device keeps resident
 *                         for the kernel instance (several per CU for small
 *                         instances; clamped to 0..resident-1), for kernels
 *                         that run beside it: collectives, copies (same bits)
 *   "work_order"          0: hand a launch's 8x8 tiles out in band order instead of
 *                         most expensive first by a counting launch's Scene.Hit
 *                         calls (same bits)
 *   "coop_lanes"          a wave whose work queue ran dry and that holds at most
 *                         this many paths finds their hits with the whole wave
 *                         scanning every sphere, one path at a time (0: never;
 *                         default 2) (same bits)
 */
#ifndef TRAY_DEBUG_H
#define TRAY_DEBUG_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* Sets knob `name` to `value`. TRAY_ERR_INVALID_ARGUMENT for an unknown name. */
int tray_debug_set(const char *name, int64_t value);
/* Unsets knob `name`, or every knob when name is NULL. */
int tray_debug_clear(const char *name);

#ifdef __cplusplus
}
#endif

#endif /* TRAY_DEBUG_H */
