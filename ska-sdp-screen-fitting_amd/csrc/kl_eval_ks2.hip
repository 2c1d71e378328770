// kl_eval_ks2.hip -- launch_eval_pick<KS> for KS = 5, 6 (see kl_eval_impl.h).
#include "kl_eval_impl.h"

namespace sf {
SF_EVAL_INSTANTIATE(5)
SF_EVAL_INSTANTIATE(6)
}  // namespace sf
