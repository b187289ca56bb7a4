// rt_dropin.cpp — the reference-side binding of INTEGRATION.md §2, compiled (Makefile target rt_dropin)
// against include/rt_api.h and the image's real <GL/gl.h> / libGL, so the documented drop-in cannot drift
// from the header.
//
// It is the part of Hw4/MySdlApplication.cpp a maintainer edits: loadScene() (MSA:1495-1539) fills the
// flat rt_scene from the same boardMap instead of building g_scene, and draw() (MSA:1541-1563) calls
// rt_render instead of rayTraceScreen (MSA:1560) and hands the RGBA8 frame to GL with glDrawPixels.  The
// screenshot path (writePpmScreenshot, Hw4/ppm.cpp:15-25) becomes rt_write_ppm on the same bottom-up buffer.
// Everything else in the application (initScene2's dialogue, SDL loop) is unchanged.
//
// As a program (the -m gpu test drives it):  rt_dropin [--frames K] [--width W --height H] --out f.ppm
//   entries...   where each entry is "<square>:<type letter>" with initScene2's letters
//                (a light, b tetrahedron, c cube, d sphere, e cylinder, f cone), e.g.  b6:a d7:d b4:b a7:c
// Without a GL context (no window here) the GL calls are no-ops of the real libGL; the frame goes to the PPM.
#include <GL/gl.h>

#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <map>
#include <stdexcept>
#include <string>
#include <vector>

#include "../../include/rt_api.h"

using namespace std;

// ---- the application's globals that the binding touches (MSA:48, 570, boardMap :1467) ---------------------
static const int MAX_DEPTH = 5;
static int g_windowWidth = 500;
static int g_windowHeight = 500;
static map<string, int> boardMap;                       // square -> {LIGHT, TETRAHEDRON, CUBE, SPHERE, CYLINDER, CONE}

// ---- the binding -----------------------------------------------------------------------
static rt_ctx* g_rt = nullptr;
static rt_scene g_rtScene;
static rt_sphere g_rtSpheres[RT_MAX_SPHERES];
static rt_mesh g_rtMeshes[RT_MAX_MESHES];
static rt_light g_rtLight;
static vector<uint8_t> g_rgba;                          // the last frame, bottom-up RGBA8 (glReadPixels layout)

void loadScene()                                        // MSA:1495 — same boardMap, now flattened
{
   vector<const char*> sq; vector<int32_t> ty;
   for (auto& kv : boardMap) { sq.push_back(kv.first.c_str()); ty.push_back(kv.second); }
   int rc = rt_load_scene(sq.data(), ty.data(), (int)sq.size(), &g_rtScene, g_rtSpheres, RT_MAX_SPHERES,
                          g_rtMeshes, RT_MAX_MESHES, &g_rtLight);
   if (rc != RT_OK) throw runtime_error(rt_last_error());
   if (!g_rt && rt_ctx_create(0, &g_rt) != RT_OK) throw runtime_error(rt_last_error());
}

void draw()                                             // MSA:1541
{
   glClear(GL_COLOR_BUFFER_BIT);
   rt_camera cam;
   rt_camera_init_reference(&cam, g_windowWidth, g_windowHeight, 1.0);   // unit pixel step, as MSA:1315
   g_rgba.resize(size_t(g_windowWidth) * g_windowHeight * 4);
   if (rt_render(g_rt, &g_rtScene, &cam, g_windowWidth, g_windowHeight, MAX_DEPTH,
                 nullptr, nullptr, g_rgba.data(), nullptr, nullptr) != RT_OK)
      throw runtime_error(rt_last_error());
   glRasterPos2i(0, 0);                                 // gluOrtho2D(0,W,0,H): bottom-left origin
   glDrawPixels(g_windowWidth, g_windowHeight, GL_RGBA, GL_UNSIGNED_BYTE, g_rgba.data());
   glFlush();
}

void writePpmScreenshot(const int width, const int height, const char* filename)   // Hw4/ppm.cpp:15
{
   if (rt_write_ppm(filename, g_rgba.data(), width, height, 4) != RT_OK) throw runtime_error(rt_last_error());
}

// ---- test driver ---------------------------------------------------------------------------------------------
int main(int argc, char** argv) {
   int frames = 1;
   string out = "dropin.ppm";
   for (int i = 1; i < argc; ++i) {
      string a = argv[i];
      if (a == "--frames" && i + 1 < argc) frames = atoi(argv[++i]);
      else if (a == "--width" && i + 1 < argc) g_windowWidth = atoi(argv[++i]);
      else if (a == "--height" && i + 1 < argc) g_windowHeight = atoi(argv[++i]);
      else if (a == "--out" && i + 1 < argc) out = argv[++i];
      else {
         size_t c = a.find(':');
         if (c == string::npos || c + 2 != a.size() || a[c + 1] < 'a' || a[c + 1] > 'f') {
            fprintf(stderr, "usage: rt_dropin [--frames K] [--width W --height H] [--out f.ppm] square:type...\n");
            return 2;
         }
         boardMap[a.substr(0, c)] = a[c + 1] - 'a';     // boardMap[tmp] = type (MSA:1467)
      }
   }
   try {
      loadScene();
      draw();                                           // first frame: scene upload, first render of the view
      const auto t0 = chrono::steady_clock::now();
      for (int k = 1; k < frames; ++k) draw();          // steady state: what the SDL loop repeats per frame
      const double ms = frames > 1 ? chrono::duration<double, milli>(chrono::steady_clock::now() - t0).count() /
                                         (frames - 1) : 0.0;
      writePpmScreenshot(g_windowWidth, g_windowHeight, out.c_str());
      printf("rt_dropin: %dx%d, %d frame(s), %.3f ms per draw() after the first -> %s\n", g_windowWidth,
             g_windowHeight, frames, ms, out.c_str());
   } catch (const exception& e) {
      fprintf(stderr, "rt_dropin: %s\n", e.what());
      return 1;
   }
   rt_ctx_destroy(g_rt);
   return 0;
}
