// kl_eval_ks3.hip -- launch_eval_pick<KS> for KS = 7, 8, 9 (see kl_eval_impl.h).
#include "kl_eval_impl.h"

namespace sf {
SF_EVAL_INSTANTIATE(7)
SF_EVAL_INSTANTIATE(8)
SF_EVAL_INSTANTIATE(9)
}  // namespace sf
