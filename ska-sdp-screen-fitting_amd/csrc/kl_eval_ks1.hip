// kl_eval_ks1.hip -- launch_eval_pick<KS> for KS = 1, 2, 3, 4 (see kl_eval_impl.h).
#include "kl_eval_impl.h"

namespace sf {
SF_EVAL_INSTANTIATE(1)
SF_EVAL_INSTANTIATE(2)
SF_EVAL_INSTANTIATE(3)
SF_EVAL_INSTANTIATE(4)
}  // namespace sf
