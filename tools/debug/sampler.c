/* sampler.c -- a SIGPROF sampling profiler for host C code running under CPython (no perf on
 * the boxes): start(us) arms a CLOCK_MONOTONIC timer, the handler records the interrupted instruction
 * pointer; stop() returns them as a list of ints; tools/debug/csample.py resolves them
 * (dladdr for the library and symbol, addr2line for lines in our own .so).  x86-64 Linux only.
 *   gcc -O2 -shared -fPIC -I<python include> tools/debug/sampler.c -o tools/debug/_sampler.so */
#define PY_SSIZE_T_CLEAN
#define _GNU_SOURCE
#include <Python.h>
#include <signal.h>
#include <string.h>
#include <sys/syscall.h>
#include <time.h>
#include <ucontext.h>
#include <unistd.h>

#define CAP (1 << 22)
static unsigned long long* g_pc;
static volatile long g_n;
static timer_t g_timer;
static int g_armed;

static void on_prof(int sig, siginfo_t* si, void* uc) {
  (void)sig;
  (void)si;
  const long i = g_n;
  if (i < CAP) {
    g_pc[i] = (unsigned long long)((ucontext_t*)uc)->uc_mcontext.gregs[REG_RIP];
    g_n = i + 1;
  }
}

static PyObject* start(PyObject* self, PyObject* args) {
  long us;
  (void)self;
  if (!PyArg_ParseTuple(args, "l", &us)) return NULL;
  if (!g_pc && !(g_pc = malloc(CAP * sizeof *g_pc))) return PyErr_NoMemory();
  g_n = 0;
  struct sigaction sa;
  memset(&sa, 0, sizeof sa);
  sa.sa_sigaction = on_prof;
  sa.sa_flags = SA_SIGINFO | SA_RESTART;
  sigemptyset(&sa.sa_mask);
  if (sigaction(SIGPROF, &sa, NULL)) return PyErr_SetFromErrno(PyExc_OSError);
  /* (a CLOCK_MONOTONIC timer signalling this thread: ITIMER_PROF ticks at the kernel's HZ) */
  struct sigevent sev;
  memset(&sev, 0, sizeof sev);
  sev.sigev_notify = SIGEV_THREAD_ID;
  sev.sigev_signo = SIGPROF;
  sev._sigev_un._tid = (int)syscall(SYS_gettid);
  if (timer_create(CLOCK_MONOTONIC, &sev, &g_timer)) return PyErr_SetFromErrno(PyExc_OSError);
  g_armed = 1;
  struct itimerspec it = {{0, us * 1000}, {0, us * 1000}};
  if (timer_settime(g_timer, 0, &it, NULL)) return PyErr_SetFromErrno(PyExc_OSError);
  Py_RETURN_NONE;
}

static PyObject* stop(PyObject* self, PyObject* noargs) {
  (void)self;
  (void)noargs;
  if (g_armed) {
    timer_delete(g_timer);
    g_armed = 0;
  }
  signal(SIGPROF, SIG_IGN);
  PyObject* l = PyList_New(g_n);
  for (long i = 0; l && i < g_n; i++) PyList_SET_ITEM(l, i, PyLong_FromUnsignedLongLong(g_pc[i]));
  return l;
}

static PyMethodDef M[] = {{"start", start, METH_VARARGS, ""}, {"stop", stop, METH_NOARGS, ""}, {NULL, NULL, 0, NULL}};
static struct PyModuleDef MOD = {PyModuleDef_HEAD_INIT, "_sampler", NULL, -1, M, NULL, NULL, NULL, NULL};
PyMODINIT_FUNC PyInit__sampler(void) { return PyModule_Create(&MOD); }
