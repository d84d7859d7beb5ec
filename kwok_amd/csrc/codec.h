// codec.h - the host codec's internal interface to the engine (codec.cpp)
#pragma once
#include "../../include/kwok_engine.h"
#include "device.h"

namespace kwok {
// the codec's compiled selectors in the device scanner's layout (json.hip)
int codec_export(const kwok_codec* c, JsonCfg* out);
}  // namespace kwok
