// rt_dropin.cpp — the reference-side binding of INTEGRATION.md §2, compiled (Makefile target rt_dropin)
// against include/rt_api.h and the image's real <GL/gl.h> / libGL, so the documented drop-in cannot drift
// from the header.
//
// It is the part of Hw4/MySdlApplication.cpp a maintainer edits: loadScene() (MSA:1495-1539) fills the
// flat rt_scene from the same boardMap instead of building g_scene, and draw() (MSA:1541-1563) calls
// rt_render_packed instead of rayTraceScreen (MSA:1560) and hands the frame to GL with glDrawPixels.  The
// screenshot path (writePpmScreenshot, Hw4/ppm.cpp:15-25) becomes rt_write_ppm on the same bottom-up buffer.
// Everything else in the application (initScene2's dialogue, SDL loop) is unchanged.
//
// The frame crosses PCIe in the narrowest exact format: GL_LUMINANCE (1 B/px) when the scene is achromatic
// (rt_scene_achromatic: the app's boards without the red cube), GL_RGB (3 B/px) otherwise, into pinned host
// memory (rt_host_alloc).  --pipelined draws the previous frame while the next one renders
// (rt_render_packed_async: one frame of latency, the copy of frame k overlaps the render of frame k+1).
//
// As a program (the -m gpu test and bench.py drive it):
//   rt_dropin [--frames K] [--width W --height H] [--pitch P] [--depth D] [--format auto|rgba|rgb|gray]
//             [--pageable] [--pipelined] --out f.ppm  entries...
//   where each entry is "<square>:<type letter>" with initScene2's letters
//   (a light, b tetrahedron, c cube, d sphere, e cylinder, f cone), e.g.  b6:a d7:d b4:b a7:c
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
static int MAX_DEPTH = 5;
static int g_windowWidth = 500;
static int g_windowHeight = 500;
static map<string, int> boardMap;                       // square -> {LIGHT, TETRAHEDRON, CUBE, SPHERE, CYLINDER, CONE}

// ---- the binding -----------------------------------------------------------------------
static rt_ctx* g_rt = nullptr;
static rt_scene g_rtScene;
static rt_sphere g_rtSpheres[RT_MAX_SPHERES];
static rt_mesh g_rtMeshes[RT_MAX_MESHES];
static rt_light g_rtLight;
static int g_format = RT_PIXEL_RGB8;                    // what crosses PCIe (loadScene picks it)
static GLenum g_glFormat = GL_RGB;
static int g_channels = 3;
static double g_pitch = 1.0;                            // unit pixel step, as MSA:1315
static bool g_pinned = true, g_pipelined = false;
static uint8_t* g_frame[2] = {nullptr, nullptr};        // bottom-up frames (glReadPixels layout)
static size_t g_frameBytes = 0;
static uint64_t g_ticket[2] = {0, 0};
static int g_shown = -1;                                // the buffer glDrawPixels last showed

static void check(int rc) {
   if (rc != RT_OK) throw runtime_error(rt_last_error());
}

static void set_format(int fmt) {
   g_format = fmt;
   g_glFormat = fmt == RT_PIXEL_GRAY8 ? GL_LUMINANCE : fmt == RT_PIXEL_RGB8 ? GL_RGB : GL_RGBA;
   check(rt_pixel_bytes(fmt, &g_channels));
}

void loadScene(const string& format)                    // MSA:1495 — same boardMap, now flattened
{
   vector<const char*> sq; vector<int32_t> ty;
   for (auto& kv : boardMap) { sq.push_back(kv.first.c_str()); ty.push_back(kv.second); }
   check(rt_load_scene(sq.data(), ty.data(), (int)sq.size(), &g_rtScene, g_rtSpheres, RT_MAX_SPHERES,
                       g_rtMeshes, RT_MAX_MESHES, &g_rtLight));
   int achromatic = 0;
   check(rt_scene_achromatic(&g_rtScene, &achromatic));
   if (format == "rgba") set_format(RT_PIXEL_RGBA8);
   else if (format == "rgb") set_format(RT_PIXEL_RGB8);
   else if (format == "gray") set_format(RT_PIXEL_GRAY8);
   else set_format(achromatic ? RT_PIXEL_GRAY8 : RT_PIXEL_RGB8);
   if (!g_rt) check(rt_ctx_create(0, &g_rt));
}

static void frame_buffers() {
   const size_t bytes = size_t(g_windowWidth) * g_windowHeight * g_channels;
   if (bytes == g_frameBytes) return;
   if (g_rt) check(rt_ctx_wait(g_rt, 0));               // (reshape) no copy may still target the old buffers
   for (auto& f : g_frame) {
      if (g_pinned) rt_host_free(f); else free(f);
      f = nullptr;
      if (g_pinned) check(rt_host_alloc(bytes, (void**)&f));
      else if (!(f = (uint8_t*)malloc(bytes))) throw runtime_error("out of memory");
   }
   g_frameBytes = bytes;
}

static void show(int b) {
   glRasterPos2i(0, 0);                                 // gluOrtho2D(0,W,0,H): bottom-left origin
   glPixelStorei(GL_UNPACK_ALIGNMENT, 1);               // rows of 1 or 3 bytes per pixel are not 4-aligned
   glDrawPixels(g_windowWidth, g_windowHeight, g_glFormat, GL_UNSIGNED_BYTE, g_frame[b]);
   glFlush();
   g_shown = b;
}

void draw()                                             // MSA:1541
{
   static uint64_t k = 0;
   glClear(GL_COLOR_BUFFER_BIT);
   rt_camera cam;
   rt_camera_init_reference(&cam, g_windowWidth, g_windowHeight, g_pitch);
   frame_buffers();
   const int b = (int)(k++ & 1);
   if (!g_pipelined) {                                  // this frame, now
      check(rt_render_packed(g_rt, &g_rtScene, &cam, g_windowWidth, g_windowHeight, MAX_DEPTH, g_format,
                             g_frame[b], nullptr));
      show(b);
      return;
   }
   // pipelined: queue this frame, then show the previous one (complete once its ticket is waited for)
   check(rt_render_packed_async(g_rt, &g_rtScene, &cam, g_windowWidth, g_windowHeight, MAX_DEPTH, g_format,
                                g_frame[b], &g_ticket[b]));
   if (k > 1) {
      check(rt_ctx_wait(g_rt, g_ticket[b ^ 1]));
      show(b ^ 1);
   }
}

void writePpmScreenshot(const int width, const int height, const char* filename)   // Hw4/ppm.cpp:15
{
   if (g_pipelined) {                                   // the last queued frame
      check(rt_ctx_wait(g_rt, 0));
      g_shown = g_ticket[0] > g_ticket[1] ? 0 : 1;
   }
   check(rt_write_ppm(filename, g_frame[g_shown], width, height, g_channels));
}

// ---- test driver ---------------------------------------------------------------------------------------------
int main(int argc, char** argv) {
   int frames = 1;
   string out = "dropin.ppm", format = "auto";
   for (int i = 1; i < argc; ++i) {
      string a = argv[i];
      if (a == "--frames" && i + 1 < argc) frames = atoi(argv[++i]);
      else if (a == "--width" && i + 1 < argc) g_windowWidth = atoi(argv[++i]);
      else if (a == "--height" && i + 1 < argc) g_windowHeight = atoi(argv[++i]);
      else if (a == "--pitch" && i + 1 < argc) g_pitch = atof(argv[++i]);
      else if (a == "--depth" && i + 1 < argc) MAX_DEPTH = atoi(argv[++i]);
      else if (a == "--format" && i + 1 < argc) format = argv[++i];
      else if (a == "--pageable") g_pinned = false;
      else if (a == "--pipelined") g_pipelined = true;
      else if (a == "--out" && i + 1 < argc) out = argv[++i];
      else {
         size_t c = a.find(':');
         if (c == string::npos || c + 2 != a.size() || a[c + 1] < 'a' || a[c + 1] > 'f') {
            fprintf(stderr, "usage: rt_dropin [--frames K] [--width W --height H] [--pitch P] [--depth D] "
                            "[--format auto|rgba|rgb|gray] [--pageable] [--pipelined] [--out f.ppm] square:type...\n");
            return 2;
         }
         boardMap[a.substr(0, c)] = a[c + 1] - 'a';     // boardMap[tmp] = type (MSA:1467)
      }
   }
   try {
      loadScene(format);
      // the first frames: scene upload and first render of the view, then the calibration render that times its tile
      // rows (rt_render_dev's adaptive order) — not the steady state the SDL loop repeats
      const int warm = frames > 3 ? 3 : 1;
      for (int k = 0; k < warm; ++k) draw();
      const auto t0 = chrono::steady_clock::now();
      for (int k = warm; k < frames; ++k) draw();      // steady state: what the SDL loop repeats per frame
      const double ms = frames > warm ? chrono::duration<double, milli>(chrono::steady_clock::now() - t0).count() /
                                            (frames - warm) : 0.0;
      writePpmScreenshot(g_windowWidth, g_windowHeight, out.c_str());
      printf("rt_dropin: %dx%d, %d frame(s), %.3f ms per draw() after the first %d, format %s (%d B/px), %s%s -> %s\n",
             g_windowWidth, g_windowHeight, frames, ms, warm,
             g_format == RT_PIXEL_GRAY8 ? "GRAY8" : g_format == RT_PIXEL_RGB8 ? "RGB8" : "RGBA8", g_channels,
             g_pinned ? "pinned" : "pageable", g_pipelined ? ", pipelined" : "", out.c_str());
   } catch (const exception& e) {
      fprintf(stderr, "rt_dropin: %s\n", e.what());
      return 1;
   }
   rt_ctx_wait(g_rt, 0);
   for (auto f : g_frame) {
      if (g_pinned) rt_host_free(f); else free(f);
   }
   rt_ctx_destroy(g_rt);
   return 0;
}
