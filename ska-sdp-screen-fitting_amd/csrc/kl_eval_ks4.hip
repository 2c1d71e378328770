// kl_eval_ks4.hip -- launch_eval_pick<KS> for KS = 10, 11, 12 (see kl_eval_impl.h).
#include "kl_eval_impl.h"

namespace sf {
SF_EVAL_INSTANTIATE(10)
SF_EVAL_INSTANTIATE(11)
SF_EVAL_INSTANTIATE(12)
}  // namespace sf
