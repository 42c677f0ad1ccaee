// Internal helpers shared by the C-ABI translation units.
#pragma once

#include <string>

namespace tray {

// Records `msg` as tray_last_error() for the calling thread and returns `code`.
int fail(int code, const std::string& msg);

}  // namespace tray
