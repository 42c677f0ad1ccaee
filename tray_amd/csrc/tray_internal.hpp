// Internal helpers shared by the C-ABI translation units.
#pragma once

#include <stdint.h>

#include <string>

namespace tray {

// Records `msg` as tray_last_error() for the calling thread and returns `code`.
int fail(int code, const std::string& msg);

// TRAY_OK when `device` is a visible gfx950 device (first use: its one-time
// setup, tray_abi.hip), else the tray_status and tray_last_error().
int device_usable(int32_t device);

// ColorF.ToSRGBA's channel encoder on the host (ray/vec3.go:173-180).
uint8_t srgb8(double c);
// The device encoder's table (tray_host.cpp): t[k], k = 1..255, is the smallest
// double c with srgb8(c) >= k (t[0] is unused). srgb8(c) is the number of
// thresholds <= c, which is how the device encodes, bit-identical by construction.
const double* srgb_thresholds();

// Test and A/B knobs (include/tray_debug.h), set only through tray_debug_set:
// the library never reads the process environment.
enum DebugKnob {
    kKnobAccSlots,
    kKnobBandSamples,
    kKnobBvhLeaf,
    kKnobBvhLdsMode,
    kKnobStackLdsSlots,
    kKnobNodeDeep,
    kKnobPrimaryCandidates,
    kKnobResolveStaged,
    kKnobWaveChunks,
    kKnobSceneContexts,
    kKnobGridReserve,
    kKnobWorkOrder,
    kKnobCoopLanes,
    kKnobCount
};
// True, with the value in *v, when the knob is set.
bool debug_knob(DebugKnob k, long long* v);

// tray_scale.hip: free the pinned tap-table staging buffers whose copies have
// completed (tray_shutdown).
void scale_release_staging();

}  // namespace tray
