// One compiled model configuration: built once per entry of the prebuilt list
// (ude_amd/configs.py) or on demand for an unlisted one (JIT), each into its
// own object, all linked into one libude_rk4*.so with ude_rk4.hip.
//   -DUDE_CFG_ID=<n> -DUDE_ONE_CONFIG=R,L,KIND,NPH,P0,P1,P2,P3,NAH,A0,A1,A2,A3
#include "ude_entry.h"

#define UDE_CAT2(a, b) a##b
#define UDE_CAT(a, b) UDE_CAT2(a, b)
#define UDE_MODEL_X(...) ude::Model<__VA_ARGS__>

// Referencing the kernels from host code instantiates them for the device pass
// as well; the registry entry itself is host data.
#if !defined(__HIP_DEVICE_COMPILE__)
namespace ude {
extern const Entry UDE_CAT(ude_entry_, UDE_CFG_ID);
const Entry UDE_CAT(ude_entry_, UDE_CFG_ID) = make_entry<UDE_MODEL_X(UDE_ONE_CONFIG)>();
}  // namespace ude
#else
template struct ude::Ops<UDE_MODEL_X(UDE_ONE_CONFIG)>;
template struct ude::DopriOps<UDE_MODEL_X(UDE_ONE_CONFIG)>;
template struct ude::LossOps<UDE_MODEL_X(UDE_ONE_CONFIG)>;
template struct ude::EvalOps<UDE_MODEL_X(UDE_ONE_CONFIG)>;
#endif
