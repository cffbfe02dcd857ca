/*
 * _scgpu_fast: a METH_FASTCALL CPython binding of the per-step C-ABI entry points
 * (scg_bg_step, scg_sc_step) so a Python step loop pays ~0.2 us of call overhead
 * instead of ctypes' argument marshalling. It links libscgpu.so (the C ABI of
 * include/scgpu.h) and adds no logic: arguments are the integer addresses of the
 * ctypes config/state structs and the tensors' data_ptr()s.
 *
 * Return value: (status << 1) | done; status != 0 is turned into the mapped Python
 * exception by the caller (gym_supplychain_amd._native.check).
 *
 * Plus node_barrier, the host barrier of bench.py's ranks on one node (below).
 */
#define PY_SSIZE_T_CLEAN
#include <Python.h>
#include <stdint.h>
#include <time.h>

#include "scgpu.h"

static int as_ptr(PyObject* o, void** out) {
  if (o == Py_None) {
    *out = NULL;
    return 0;
  }
  unsigned long long v = PyLong_AsUnsignedLongLong(o);
  if (v == (unsigned long long)-1 && PyErr_Occurred()) return -1;
  *out = (void*)(uintptr_t)v;
  return 0;
}

/* bg_step(cfg, state, action, obs, reward, terminal_obs, flags, stream) */
static PyObject* bg_step(PyObject* self, PyObject* const* args, Py_ssize_t nargs) {
  (void)self;
  void* p[8];
  if (nargs != 8) {
    PyErr_SetString(PyExc_TypeError, "bg_step expects 8 arguments");
    return NULL;
  }
  for (int i = 0; i < 8; ++i)
    if (as_ptr(args[i], &p[i])) return NULL;
  int32_t done = 0;
  const int rc = scg_bg_step((const scg_bg_config*)p[0], (scg_bg_state*)p[1], (const int32_t*)p[2], (int32_t*)p[3],
                             (int32_t*)p[4], (int32_t*)p[5], (uint32_t)(uintptr_t)p[6], &done, p[7]);
  return PyLong_FromLong((long)((rc << 1) | (done ? 1 : 0)));
}

/* A vec env's fixed step arguments, filled once by the Python side (its address is the
 * handle): bg_step_h(handle, action, stream) then parses three arguments per step. */
typedef struct bg_step_args {
  uint64_t cfg, state, obs, reward, terminal_obs;
  uint32_t flags;
} bg_step_args;

/* bg_step_h(handle, action, stream) */
static PyObject* bg_step_h(PyObject* self, PyObject* const* args, Py_ssize_t nargs) {
  (void)self;
  void* p[3];
  if (nargs != 3) {
    PyErr_SetString(PyExc_TypeError, "bg_step_h expects 3 arguments");
    return NULL;
  }
  for (int i = 0; i < 3; ++i)
    if (as_ptr(args[i], &p[i])) return NULL;
  const bg_step_args* h = (const bg_step_args*)p[0];
  if (!h) {
    PyErr_SetString(PyExc_ValueError, "bg_step_h: null handle");
    return NULL;
  }
  int32_t done = 0;
  const int rc = scg_bg_step((const scg_bg_config*)(uintptr_t)h->cfg, (scg_bg_state*)(uintptr_t)h->state,
                             (const int32_t*)p[1], (int32_t*)(uintptr_t)h->obs, (int32_t*)(uintptr_t)h->reward,
                             (int32_t*)(uintptr_t)h->terminal_obs, h->flags, &done, p[2]);
  return PyLong_FromLong((long)((rc << 1) | (done ? 1 : 0)));
}

/* bg_step_timed(cfg, state, action, obs, reward, terminal_obs, flags, start_event, stop_event, stream) */
static PyObject* bg_step_timed(PyObject* self, PyObject* const* args, Py_ssize_t nargs) {
  (void)self;
  void* p[10];
  if (nargs != 10) {
    PyErr_SetString(PyExc_TypeError, "bg_step_timed expects 10 arguments");
    return NULL;
  }
  for (int i = 0; i < 10; ++i)
    if (as_ptr(args[i], &p[i])) return NULL;
  int32_t done = 0;
  const int rc = scg_bg_step_timed((const scg_bg_config*)p[0], (scg_bg_state*)p[1], (const int32_t*)p[2],
                                   (int32_t*)p[3], (int32_t*)p[4], (int32_t*)p[5], (uint32_t)(uintptr_t)p[6], &done,
                                   p[7], p[8], p[9]);
  return PyLong_FromLong((long)((rc << 1) | (done ? 1 : 0)));
}

/* bg_server_step(cfg, state, slot): one week through the step server — post, spin up to
 * 200 us holding the GIL (the answer usually comes in a few), then wait with the GIL released
 * (other Python threads run; the C wait fails after 60 s or on a HIP error of the wave's stream). */
static PyObject* bg_server_step(PyObject* self, PyObject* const* args, Py_ssize_t nargs) {
  (void)self;
  void* p[3];
  if (nargs != 3) {
    PyErr_SetString(PyExc_TypeError, "bg_server_step expects 3 arguments");
    return NULL;
  }
  for (int i = 0; i < 3; ++i)
    if (as_ptr(args[i], &p[i])) return NULL;
  scg_bg_state* st = (scg_bg_state*)p[1];
  scg_bg_server_slot* slot = (scg_bg_server_slot*)p[2];
  int32_t done = 0;
  int rc = scg_bg_server_post((const scg_bg_config*)p[0], st, slot);
  if (rc == SCG_OK) rc = scg_bg_server_wait(st, slot, 200, &done);
  if (rc == SCG_PENDING) {
    Py_BEGIN_ALLOW_THREADS
    rc = scg_bg_server_wait(st, slot, -1, &done);
    Py_END_ALLOW_THREADS
  }
  return PyLong_FromLong((long)((rc << 1) | (done ? 1 : 0)));
}

/* sc_server_step(cfg, state, server): one step through the SupplyChain step server, as
 * bg_server_step (post, spin up to 200 us with the GIL, then wait without it). */
static PyObject* sc_server_step(PyObject* self, PyObject* const* args, Py_ssize_t nargs) {
  (void)self;
  void* p[3];
  if (nargs != 3) {
    PyErr_SetString(PyExc_TypeError, "sc_server_step expects 3 arguments");
    return NULL;
  }
  for (int i = 0; i < 3; ++i)
    if (as_ptr(args[i], &p[i])) return NULL;
  const scg_sc_config* cfg = (const scg_sc_config*)p[0];
  scg_sc_state* st = (scg_sc_state*)p[1];
  scg_sc_server* sv = (scg_sc_server*)p[2];
  int32_t done = 0;
  int rc = scg_sc_server_post(cfg, st, sv);
  if (rc == SCG_OK) rc = scg_sc_server_wait(cfg, st, sv, 200, &done);
  if (rc == SCG_PENDING) {
    Py_BEGIN_ALLOW_THREADS
    rc = scg_sc_server_wait(cfg, st, sv, -1, &done);
    Py_END_ALLOW_THREADS
  }
  return PyLong_FromLong((long)((rc << 1) | (done ? 1 : 0)));
}

/* sc_step(cfg, state, action, obs, reward, terminal_obs, flags, stream) */
static PyObject* sc_step(PyObject* self, PyObject* const* args, Py_ssize_t nargs) {
  (void)self;
  void* p[8];
  if (nargs != 8) {
    PyErr_SetString(PyExc_TypeError, "sc_step expects 8 arguments");
    return NULL;
  }
  for (int i = 0; i < 8; ++i)
    if (as_ptr(args[i], &p[i])) return NULL;
  int32_t done = 0;
  const int rc = scg_sc_step((const scg_sc_config*)p[0], (scg_sc_state*)p[1], (const float*)p[2], p[3],
                             (double*)p[4], p[5], (uint32_t)(uintptr_t)p[6], &done, p[7]);
  return PyLong_FromLong((long)((rc << 1) | (done ? 1 : 0)));
}

static int64_t now_us(void) {
  struct timespec ts;
  clock_gettime(CLOCK_MONOTONIC, &ts);
  return (int64_t)ts.tv_sec * 1000000 + ts.tv_nsec / 1000;
}

/* node_barrier(words, world, sense, timeout_us) -> the new sense. A sense-reversing barrier
 * of `world` processes of one node on two int32 words of a shared page: words[0] counts
 * arrivals, words[1] is the phase. Every rank passes its last returned sense (0 at first);
 * the last to arrive resets the count and flips the phase, the others spin until it flips.
 * TimeoutError after timeout_us (a rank that never comes). The GIL is released while
 * waiting. A timed-out call leaves its arrival counted and the caller's sense unchanged, so
 * the page is unusable afterwards (bench.NodeBarrier drops it). */
static PyObject* node_barrier(PyObject* self, PyObject* const* args, Py_ssize_t nargs) {
  (void)self;
  void* p;
  if (nargs != 4) {
    PyErr_SetString(PyExc_TypeError, "node_barrier expects 4 arguments");
    return NULL;
  }
  if (as_ptr(args[0], &p)) return NULL;
  const long world = PyLong_AsLong(args[1]);
  const long old = PyLong_AsLong(args[2]);
  const long long timeout_us = PyLong_AsLongLong(args[3]);
  if (PyErr_Occurred()) return NULL;
  if (!p || world < 1) {
    PyErr_SetString(PyExc_ValueError, "node_barrier: null page or world < 1");
    return NULL;
  }
  int32_t* w = (int32_t*)p;
  const int32_t sense = old ? 0 : 1;
  int timed_out = 0;
  Py_BEGIN_ALLOW_THREADS
  if (__atomic_fetch_add(&w[0], 1, __ATOMIC_ACQ_REL) == world - 1) {
    __atomic_store_n(&w[0], 0, __ATOMIC_RELAXED);
    __atomic_store_n(&w[1], sense, __ATOMIC_RELEASE);
  } else {
    const int64_t t0 = now_us();
    unsigned spins = 0;
    while (__atomic_load_n(&w[1], __ATOMIC_ACQUIRE) != sense) {
      if ((++spins & 1023u) == 0 && now_us() - t0 > timeout_us) {
        timed_out = 1;
        break;
      }
      __builtin_ia32_pause();
    }
  }
  Py_END_ALLOW_THREADS
  if (timed_out) {
    PyErr_SetString(PyExc_TimeoutError, "node_barrier: not every rank arrived");
    return NULL;
  }
  return PyLong_FromLong(sense);
}

static PyMethodDef methods[] = {
    {"bg_step", (PyCFunction)(void (*)(void))bg_step, METH_FASTCALL, "scg_bg_step"},
    {"bg_step_h", (PyCFunction)(void (*)(void))bg_step_h, METH_FASTCALL, "scg_bg_step with the fixed arguments behind a handle"},
    {"bg_server_step", (PyCFunction)(void (*)(void))bg_server_step, METH_FASTCALL, "scg_bg_server_step"},
    {"bg_step_timed", (PyCFunction)(void (*)(void))bg_step_timed, METH_FASTCALL, "scg_bg_step_timed"},
    {"sc_step", (PyCFunction)(void (*)(void))sc_step, METH_FASTCALL, "scg_sc_step"},
    {"sc_server_step", (PyCFunction)(void (*)(void))sc_server_step, METH_FASTCALL, "scg_sc_server_post + _wait"},
    {"node_barrier", (PyCFunction)(void (*)(void))node_barrier, METH_FASTCALL, "host barrier of one node's ranks"},
    {NULL, NULL, 0, NULL},
};

static struct PyModuleDef module = {PyModuleDef_HEAD_INIT, "_scgpu_fast", NULL, -1, methods,
                                    NULL, NULL, NULL, NULL};

PyMODINIT_FUNC PyInit__scgpu_fast(void) { return PyModule_Create(&module); }
