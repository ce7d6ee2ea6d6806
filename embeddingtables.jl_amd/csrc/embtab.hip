// embtab.hip — unity translation unit of libembtab_hip.so (gfx950 only).
// One TU so the device-side error counter (et::g_oob_count) is shared by every
// kernel without relocatable device code.
#include "et_common.h"
#include "et_lookup.hip"
#include "et_update.hip"
#include "et_misc.hip"
