// rt_render_b1.hip — the depth-1 instances of the render and ray-list kernels (rt_render.hpp).  One
// translation unit per depth: the eight depths compile in parallel.
#include "rt_render.hpp"

RT_RENDER_INSTANCES(1)
