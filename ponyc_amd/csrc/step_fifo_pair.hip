// k_step for engines whose serial actors are FIFO sources and sinks (the
// table pair zone_dev.h kHtFifoPair) (step_tu.h).
#define GPA_STEP_HT 64
#define GPA_STEP_ENTRY step_entry_fifo_pair
#include "step_tu.h"
