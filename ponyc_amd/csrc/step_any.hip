// k_step for any mix of handler tables (a switch over the actor's table) (step_tu.h).
#define GPA_STEP_HT -1
#define GPA_STEP_ENTRY step_entry_any
#include "step_tu.h"
