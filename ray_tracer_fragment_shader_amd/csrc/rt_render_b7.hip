// rt_render_b7.hip — the depth-7 instances of the render and ray-list kernels (rt_render.hpp).  One
// translation unit per depth: the eight depths compile in parallel.
#include "rt_render.hpp"

RT_RENDER_INSTANCES(7)
