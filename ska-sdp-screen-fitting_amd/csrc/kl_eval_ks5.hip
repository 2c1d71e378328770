// kl_eval_ks5.hip -- launch_eval_pick<KS> for KS = 13, 14, 15 (see kl_eval_impl.h).
#include "kl_eval_impl.h"

namespace sf {
SF_EVAL_INSTANTIATE(13)
SF_EVAL_INSTANTIATE(14)
SF_EVAL_INSTANTIATE(15)
}  // namespace sf
