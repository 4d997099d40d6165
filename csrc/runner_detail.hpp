// Helpers shared by the engine's translation units (runner.cpp, step_driver.cpp);
// not part of the engine's interface (runner.hpp).
#pragma once

#include <cstddef>
#include <vector>

#include "schedule.hpp"
#include "transport.hpp"

namespace p2p {
namespace detail {

// Receive-slot stride: the slot size rounded up to 4 KiB (every slot and
// send region starts 16-byte aligned for the copy kernel).
size_t slot_stride(size_t bytes);

// Slot on the receiver of each flow of a phase: flows were appended in the
// same order as the receiver's recv_from list (schedule.cpp add_flow).
std::vector<int> flow_slots(const Phase& phase);

// Whether rank r posts the groups of a phase: its endpoints, and with a
// multi-path transport every rank (it may relay).
bool posts_phase(const Transport& t, const Phase& phase, int r);

// P2P_INJECT_FAULT="<kind>@<rank>[:<phase>]" names this rank (and phase;
// phase_index -1 matches any).
bool fault_applies(const char* kind, int rank, long phase_index);

}  // namespace detail
}  // namespace p2p
