// ref_prelude.hpp — TEST INFRASTRUCTURE (oracle/_ref build only).
// The standard-library part of Hw4/MySdlApplication.h:9-17, which the extracted hot-path line ranges of
// Hw4/MySdlApplication.cpp need.  <SDL.h> and "glsupport.h" (GLEW) are NOT included and NOT stood in
// for: the extracted ranges (constants, Point..CheckerBoard, materials/g_scene, intersection code,
// rayTraceRay, convertStringCoordinate) use none of them.  GLdouble/GLsizei come from the image's
// real <GL/gl.h>.
#include <GL/gl.h>
#include <iostream>
#include <cmath>
#include <cstdlib>
#include <vector>
#include <string>
#include <map>
using namespace std;
