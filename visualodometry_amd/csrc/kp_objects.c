/* _vo_keypoints: the cv2.KeyPoint objects SIFT.detectAndCompute returns, built in bulk.
 *
 * The reference's front end keeps OpenCV's Python objects (frontend.py:55 detectAndCompute,
 * frontend.py:59 `k.pt` per keypoint).  Building 4000 of them one Python statement at a time
 * cost ~0.8 ms per frame on the MI355X host, two thirds of the GPU pipeline itself; this module
 * builds the tuple from the device's 32-byte keypoint records (vo_sift_keypoint, include/vo_hip.h)
 * in one C loop.
 *
 * KeyPoint mirrors cv2.KeyPoint's Python surface: the constructor KeyPoint(x, y, size, angle=-1,
 * response=0, octave=0, class_id=-1) and the attributes pt (a fresh (x, y) tuple of floats per
 * read, as OpenCV's getter), size, angle, response (float32 storage, read as Python floats),
 * octave and class_id (ints); all writable.  Host marshalling only: no GPU work here.
 */
#define PY_SSIZE_T_CLEAN
#include <Python.h>
#include <stddef.h>
#include <stdint.h>
#include <string.h>
#include <structmember.h>

typedef struct {
  PyObject_HEAD
  float x, y, size, angle, response;
  int octave, class_id;
} KeyPointObject;

/* vo_sift_keypoint: x, y, size, angle, response (f32), octave, image, reserved (i32) */
typedef struct {
  float x, y, size, angle, response;
  int32_t octave, image, reserved;
} Record;

static PyTypeObject KeyPointType;

static int kp_init(KeyPointObject* self, PyObject* args, PyObject* kw) {
  static char* names[] = {"x", "y", "size", "angle", "response", "octave", "class_id", NULL};
  double x, y, size, angle = -1.0, response = 0.0;
  int octave = 0, class_id = -1;
  if (!PyArg_ParseTupleAndKeywords(args, kw, "ddd|ddii:KeyPoint", names, &x, &y, &size, &angle, &response,
                                   &octave, &class_id))
    return -1;
  self->x = (float)x;
  self->y = (float)y;
  self->size = (float)size;
  self->angle = (float)angle;
  self->response = (float)response;
  self->octave = octave;
  self->class_id = class_id;
  return 0;
}

static PyObject* kp_get_pt(KeyPointObject* self, void* closure) {
  (void)closure;
  return Py_BuildValue("(dd)", (double)self->x, (double)self->y);
}

static int kp_set_pt(KeyPointObject* self, PyObject* value, void* closure) {
  (void)closure;
  double x, y;
  if (value == NULL) {
    PyErr_SetString(PyExc_AttributeError, "KeyPoint.pt cannot be deleted");
    return -1;
  }
  if (!PyArg_ParseTuple(value, "dd:KeyPoint.pt", &x, &y)) return -1;
  self->x = (float)x;
  self->y = (float)y;
  return 0;
}

static PyObject* kp_repr(KeyPointObject* self) {
  char buf[160];
  PyOS_snprintf(buf, sizeof buf, "KeyPoint(pt=(%.9g, %.9g), size=%.9g, angle=%.9g, response=%.9g, octave=%d)",
                (double)self->x, (double)self->y, (double)self->size, (double)self->angle, (double)self->response,
                self->octave);
  return PyUnicode_FromString(buf);
}

static PyMemberDef kp_members[] = {
    {"size", T_FLOAT, offsetof(KeyPointObject, size), 0, "diameter of the keypoint's neighbourhood"},
    {"angle", T_FLOAT, offsetof(KeyPointObject, angle), 0, "orientation in degrees [0, 360)"},
    {"response", T_FLOAT, offsetof(KeyPointObject, response), 0, "|DoG| response"},
    {"octave", T_INT, offsetof(KeyPointObject, octave), 0, "OpenCV-packed octave | layer << 8 | xi"},
    {"class_id", T_INT, offsetof(KeyPointObject, class_id), 0, "object class (-1)"},
    {NULL, 0, 0, 0, NULL}};

static PyGetSetDef kp_getset[] = {{"pt", (getter)kp_get_pt, (setter)kp_set_pt, "(x, y) in pixels", NULL},
                                  {NULL, NULL, NULL, NULL, NULL}};

static PyTypeObject KeyPointType = {
    PyVarObject_HEAD_INIT(NULL, 0).tp_name = "visualodometry_amd._vo_keypoints.KeyPoint",
    .tp_basicsize = sizeof(KeyPointObject),
    .tp_flags = Py_TPFLAGS_DEFAULT,
    .tp_doc = "cv2.KeyPoint's Python surface: KeyPoint(x, y, size, angle=-1, response=0, octave=0, class_id=-1)",
    .tp_new = PyType_GenericNew,
    .tp_init = (initproc)kp_init,
    .tp_repr = (reprfunc)kp_repr,
    .tp_members = kp_members,
    .tp_getset = kp_getset,
};

/* build(records) -> tuple of KeyPoint: `records` is any C-contiguous buffer of whole
 * vo_sift_keypoint records (the KP_DTYPE numpy array of detect_and_compute). */
static PyObject* kp_build(PyObject* module, PyObject* arg) {
  (void)module;
  Py_buffer view;
  if (PyObject_GetBuffer(arg, &view, PyBUF_C_CONTIGUOUS) < 0) return NULL;
  if (view.len % (Py_ssize_t)sizeof(Record) != 0) {
    PyBuffer_Release(&view);
    PyErr_Format(PyExc_ValueError, "build: %zd bytes is not a whole number of %zu-byte keypoint records", view.len,
                 sizeof(Record));
    return NULL;
  }
  const Py_ssize_t n = view.len / (Py_ssize_t)sizeof(Record);
  PyObject* out = PyTuple_New(n);
  if (out == NULL) {
    PyBuffer_Release(&view);
    return NULL;
  }
  const char* base = (const char*)view.buf;
  for (Py_ssize_t i = 0; i < n; ++i) {
    Record r;
    memcpy(&r, base + i * (Py_ssize_t)sizeof(Record), sizeof r);
    KeyPointObject* k = PyObject_New(KeyPointObject, &KeyPointType);
    if (k == NULL) {
      Py_DECREF(out);
      PyBuffer_Release(&view);
      return NULL;
    }
    k->x = r.x;
    k->y = r.y;
    k->size = r.size;
    k->angle = r.angle;
    k->response = r.response;
    k->octave = r.octave;
    k->class_id = -1;
    PyTuple_SET_ITEM(out, i, (PyObject*)k);
  }
  PyBuffer_Release(&view);
  return out;
}

static PyMethodDef module_methods[] = {
    {"build", kp_build, METH_O, "build(records) -> tuple of KeyPoint from vo_sift_keypoint records"},
    {NULL, NULL, 0, NULL}};

static struct PyModuleDef module_def = {PyModuleDef_HEAD_INIT, "_vo_keypoints",
                                        "cv2.KeyPoint objects built in bulk from SIFT keypoint records", -1,
                                        module_methods};

PyMODINIT_FUNC PyInit__vo_keypoints(void) {
  if (PyType_Ready(&KeyPointType) < 0) return NULL;
  PyObject* m = PyModule_Create(&module_def);
  if (m == NULL) return NULL;
  Py_INCREF(&KeyPointType);
  if (PyModule_AddObject(m, "KeyPoint", (PyObject*)&KeyPointType) < 0) {
    Py_DECREF(&KeyPointType);
    Py_DECREF(m);
    return NULL;
  }
  return m;
}
