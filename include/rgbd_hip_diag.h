/* Diagnostic entry points of the DIAGNOSTIC build only (librgbd_hip_diag.so, `make -C
 * rgb-d-instance-segmentation_amd/csrc diag`, compiled with -DRGBD_DIAG).  The product library
 * (librgbd_hip.so) neither exports these nor contains the stamped kernel instantiations; the
 * tools that read them (tools/conv5_stamps.py, tools/chain_stamps.py, tools/dsam_stamps.py) load
 * the diagnostic build through RGBD_HIP_LIB. */
#ifndef RGBD_HIP_DIAG_H
#define RGBD_HIP_DIAG_H
#include "rgbd_hip.h"
#ifdef __cplusplus
extern "C" {
#endif

/* Diagnostics: buf (device, >= 2 * 12 * 8 * 5 uint64) receives, for workgroup 0 of every later
 * bf16 conv5 launch (k_rp_conv5_v4), s_memtime stamps per K step and wave of its first two items
 * (step top, after the weight-copy issue, after the first kx group + input-copy issue, after the
 * last MFMAs, after the closing wait + barrier): [item][step][wave][5]; NULL stops.  conv5's
 * timing-only variants (copies, barrier or fragment reads removed) are compile-time:
 * tools/build_variant.sh NAME -DC4_NODMA=bits. */
int rgbd_debug_conv5_stamps(void* buf);
/* The same for the bf16 chain kernels (k_rp_chain_v2 phases 0 and 1): buf (device, >= 2 * 4 * 8 * 7
 * uint64) receives workgroup 0's stamps for its tiles 8-11 (tile top, patch staged, next
 * patch issued, stem MFMAs issued, stem ReLU/pack, fusion MFMAs issued, tile end), phase-major
 * (phase 0 writes the first four points).  NULL stops. */
int rgbd_debug_chain_stamps(void* buf);
/* The same for the DSAM conv legs (k_dsam_lds, the forward cascade and dX): buf (device, >= launches
 * * 256 * 4 * 8 uint64) receives, for the next `launches` launches, per workgroup and for its first
 * four work items: s_memtime at item taken, tables built, first DMA landed, K loop done, partial
 * hand-off done, epilogue done; steps | chunks << 16 | chunk << 24; the item word.  (NULL, 0)
 * stops. */
int rgbd_debug_dsam_stamps(void* buf, int launches);
/* Timing-only variants of the stamped DSAM conv kernel (KC = 3 legs; results are garbage): mode
 * bit 0 drops the in-loop weight copies, bit 1 the in-loop input copies, bit 2 the per-step
 * barrier, bit 3 the fragment reads; bit 5 sources every step's weight copies from its code's
 * first filter tile, bit 6 every step's input copies from one fixed pixel block (L2-resident).
 * Valid: 0, 1, 2, 3, 7, 8, 15, 32, 64, 96; applies while stamps are on. */
int rgbd_debug_dsam_mode(int mode);
/* The stem statistics' lag kernel (k_stem_lag): buf (device, >= workgroups * 8 * 6 uint64)
 * receives, for every workgroup and wave of each later launch, s_memtime at entry, window staged,
 * lag loop done, waves joined, correlations written, plane sums written.  NULL stops. */
int rgbd_debug_stem_lag_stamps(void* buf);

#ifdef __cplusplus
}
#endif
#endif /* RGBD_HIP_DIAG_H */
