// emulator: the HIP runtime API lives in hip_runtime.h
#pragma once
#include "hip_runtime.h"
