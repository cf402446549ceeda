/*
 * harness.c -- TEST INFRASTRUCTURE: a JNIEnv of its own (tests/jni_harness/jni.h) and a plain C API over the natives of
 * jni/ngsep_gpu_jni.c, so tests/test_jni_shim.py can drive the shim the way the JVM would (Java strings, int[] /
 * long[] / String[] arrays, exceptions) from ctypes.  Objects are tagged heap blocks; nothing here is product code.
 */
#include <stdarg.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "jni.h"

enum { K_CLASS, K_STRING, K_INTS, K_LONGS, K_BYTES, K_DOUBLES, K_OBJS };
struct _jobject {
    int kind;
    jsize len;
    void* data;          /* string: NUL-terminated; arrays: elements */
    char name[64];       /* class name */
};

static char g_exception[1024];

static jobject make(int kind, jsize len, size_t elem) {
    jobject o = (jobject)calloc(1, sizeof(struct _jobject));
    o->kind = kind;
    o->len = len;
    o->data = calloc((size_t)(len > 0 ? len : 1), elem ? elem : 1);
    return o;
}
static void drop(jobject o) {
    if (!o) return;
    if (o->kind == K_OBJS) for (jsize i = 0; i < o->len; i++) drop(((jobject*)o->data)[i]);
    free(o->data);
    free(o);
}
static size_t elem_size(int kind) {
    switch (kind) {
        case K_INTS: return 4;
        case K_LONGS: case K_DOUBLES: return 8;
        case K_BYTES: return 1;
        case K_OBJS: return sizeof(jobject);
        default: return 1;
    }
}

static jclass e_FindClass(JNIEnv* env, const char* n) {
    (void)env;
    jobject c = make(K_CLASS, 0, 1);
    snprintf(c->name, sizeof c->name, "%s", n);
    return c;                                  /* (leaked per call: a test process) */
}
static jint e_ThrowNew(JNIEnv* env, jclass k, const char* msg) {
    (void)env;
    snprintf(g_exception, sizeof g_exception, "%s: %s", k ? k->name : "?", msg ? msg : "");
    return 0;
}
static jstring e_NewStringUTF(JNIEnv* env, const char* s) {
    (void)env;
    const size_t n = strlen(s);
    jobject o = make(K_STRING, (jsize)n, 1);
    free(o->data);
    o->data = malloc(n + 1);
    memcpy(o->data, s, n + 1);
    return o;
}
static const char* e_GetStringUTFChars(JNIEnv* env, jstring s, jboolean* copy) {
    (void)env;
    if (copy) *copy = 1;
    const size_t n = strlen((const char*)s->data);
    char* c = (char*)malloc(n + 1);
    memcpy(c, s->data, n + 1);
    return c;
}
static void e_ReleaseStringUTFChars(JNIEnv* env, jstring s, const char* c) { (void)env; (void)s; free((void*)c); }
static jsize e_GetArrayLength(JNIEnv* env, jarray a) { (void)env; return a->len; }
static jobjectArray e_NewObjectArray(JNIEnv* env, jsize n, jclass k, jobject init) {
    (void)env; (void)k; (void)init;
    return make(K_OBJS, n, sizeof(jobject));
}
static jobject e_GetObjectArrayElement(JNIEnv* env, jobjectArray a, jsize i) { (void)env; return ((jobject*)a->data)[i]; }
static void e_SetObjectArrayElement(JNIEnv* env, jobjectArray a, jsize i, jobject v) { (void)env; ((jobject*)a->data)[i] = v; }
static jbyteArray e_NewByteArray(JNIEnv* env, jsize n) { (void)env; return make(K_BYTES, n, 1); }
static jlongArray e_NewLongArray(JNIEnv* env, jsize n) { (void)env; return make(K_LONGS, n, 8); }
/* Get*Elements hand out a copy (as a JVM may), written back unless JNI_ABORT */
static void* get_copy(jarray a) {
    const size_t b = (size_t)a->len * elem_size(a->kind);
    void* c = malloc(b ? b : 1);
    memcpy(c, a->data, b);
    return c;
}
static void release_copy(jarray a, void* c, jint mode) {
    if (mode != JNI_ABORT) memcpy(a->data, c, (size_t)a->len * elem_size(a->kind));
    free(c);
}
static jint* e_GetIntArrayElements(JNIEnv* env, jintArray a, jboolean* copy) { (void)env; if (copy) *copy = 1; return (jint*)get_copy(a); }
static void e_ReleaseIntArrayElements(JNIEnv* env, jintArray a, jint* c, jint mode) { (void)env; release_copy(a, c, mode); }
static jlong* e_GetLongArrayElements(JNIEnv* env, jlongArray a, jboolean* copy) { (void)env; if (copy) *copy = 1; return (jlong*)get_copy(a); }
static void e_ReleaseLongArrayElements(JNIEnv* env, jlongArray a, jlong* c, jint mode) { (void)env; release_copy(a, c, mode); }
static void e_SetByteArrayRegion(JNIEnv* env, jbyteArray a, jsize s, jsize n, const jbyte* v) { (void)env; memcpy((jbyte*)a->data + s, v, (size_t)n); }
static void e_SetLongArrayRegion(JNIEnv* env, jlongArray a, jsize s, jsize n, const jlong* v) { (void)env; memcpy((jlong*)a->data + s, v, (size_t)n * 8); }
/* critical sections: the array's own storage (as a JVM that pins) */
static void* e_GetPrimitiveArrayCritical(JNIEnv* env, jarray a, jboolean* copy) { (void)env; if (copy) *copy = 0; return a->data; }
static void e_ReleasePrimitiveArrayCritical(JNIEnv* env, jarray a, void* c, jint mode) { (void)env; (void)a; (void)c; (void)mode; }
static jmethodID e_GetStaticMethodID(JNIEnv* env, jclass k, const char* n, const char* sig) {
    (void)env; (void)k; (void)n; (void)sig;
    return (jmethodID)(intptr_t)1;
}
/* ByteBuffer.wrap(byte[]): the array itself stands for the buffer */
static jobject e_CallStaticObjectMethod(JNIEnv* env, jclass k, jmethodID m, ...) {
    (void)env; (void)k; (void)m;
    va_list ap;
    va_start(ap, m);
    jobject arr = va_arg(ap, jobject);
    va_end(ap);
    return arr;
}

static jbyte* e_GetByteArrayElements(JNIEnv* env, jbyteArray a, jboolean* copy) { (void)env; if (copy) *copy = 1; return (jbyte*)get_copy(a); }
static void e_ReleaseByteArrayElements(JNIEnv* env, jbyteArray a, jbyte* c, jint mode) { (void)env; release_copy(a, c, mode); }
/* ByteOrder.LITTLE_ENDIAN (a static field) and ByteBuffer.order(ByteOrder): the order set is recorded */
static int g_order_le;
static jfieldID e_GetStaticFieldID(JNIEnv* env, jclass k, const char* n, const char* sig) {
    (void)env; (void)k; (void)sig;
    return (jfieldID)(intptr_t)(strcmp(n, "LITTLE_ENDIAN") == 0 ? 2 : 3);
}
static jobject e_GetStaticObjectField(JNIEnv* env, jclass k, jfieldID f) {
    (void)env; (void)k;
    static struct _jobject le = {K_CLASS, 0, NULL, "LITTLE_ENDIAN"}, be = {K_CLASS, 0, NULL, "BIG_ENDIAN"};
    return (intptr_t)f == 2 ? &le : &be;
}
static jmethodID e_GetMethodID(JNIEnv* env, jclass k, const char* n, const char* sig) {
    (void)env; (void)k; (void)n; (void)sig;
    return (jmethodID)(intptr_t)4;
}
static jobject e_CallObjectMethod(JNIEnv* env, jobject o, jmethodID m, ...) {
    (void)env; (void)m;
    va_list ap;
    va_start(ap, m);
    jobject arg = va_arg(ap, jobject);
    va_end(ap);
    g_order_le = arg && strcmp(arg->name, "LITTLE_ENDIAN") == 0;
    return o;
}

static const struct JNINativeInterface_ g_table = {
    e_FindClass, e_ThrowNew, e_NewStringUTF, e_GetStringUTFChars, e_ReleaseStringUTFChars, e_GetArrayLength,
    e_NewObjectArray, e_GetObjectArrayElement, e_SetObjectArrayElement, e_NewByteArray, e_NewLongArray,
    e_GetIntArrayElements, e_ReleaseIntArrayElements, e_GetLongArrayElements, e_ReleaseLongArrayElements,
    e_SetByteArrayRegion, e_SetLongArrayRegion, e_GetPrimitiveArrayCritical, e_ReleasePrimitiveArrayCritical,
    e_GetStaticMethodID, e_CallStaticObjectMethod, e_GetByteArrayElements, e_ReleaseByteArrayElements,
    e_GetStaticFieldID, e_GetStaticObjectField, e_GetMethodID, e_CallObjectMethod};
static JNIEnv g_env = &g_table;

/* ---- the natives (jni/ngsep_gpu_jni.c) ---- */
#define NAT(name) Java_ngsep_discovery_gpu_GpuPileupEngine_##name
jlong NAT(open)(JNIEnv*, jclass, jint, jintArray, jdouble, jstring, jstring);
void NAT(close)(JNIEnv*, jclass, jlong);
jstring NAT(lastError)(JNIEnv*, jclass, jlong);
jint NAT(loadFasta)(JNIEnv*, jclass, jlong, jstring);
jint NAT(callBam)(JNIEnv*, jclass, jlong, jstring, jstring);
jint NAT(callRegionBam)(JNIEnv*, jclass, jlong, jstring, jstring, jlong, jlong, jstring);
jint NAT(callPopulationBams)(JNIEnv*, jclass, jlong, jobjectArray, jstring);
jint NAT(callBamMulti)(JNIEnv*, jclass, jlongArray, jstring, jstring, jlong);
jint NAT(callPopulationBamsMulti)(JNIEnv*, jclass, jlongArray, jobjectArray, jstring, jlong);
jint NAT(setKnownVariants)(JNIEnv*, jclass, jlong, jstring);
jint NAT(setKnownSTRs)(JNIEnv*, jclass, jlong, jstring);
jobjectArray NAT(carvedRegions)(JNIEnv*, jclass, jlong);
jint NAT(processAlignments)(JNIEnv*, jclass, jlong, jintArray, jintArray, jintArray, jintArray, jlongArray, jintArray,
                            jintArray, jlongArray, jintArray, jbyteArray, jbyteArray, jbyteArray);
jint NAT(notifyEnd)(JNIEnv*, jclass, jlong);
jobject NAT(fetchSites)(JNIEnv*, jclass, jlong);

/* ---- a plain C API for ctypes ---- */
static jstring js(const char* s) { return s ? e_NewStringUTF(&g_env, s) : NULL; }
static jobjectArray jstrings(const char* const* v, int n) {
    jobjectArray a = make(K_OBJS, n, sizeof(jobject));
    for (int i = 0; i < n; i++) ((jobject*)a->data)[i] = js(v[i]);
    return a;
}
static jlongArray jlongs(const int64_t* v, int n) {
    jlongArray a = make(K_LONGS, n, 8);
    memcpy(a->data, v, (size_t)n * 8);
    return a;
}

const char* h_exception(void) { return g_exception; }
void h_clear_exception(void) { g_exception[0] = 0; }

int64_t h_open(int device, const int32_t* opts, int n_opts, double het, const char* qseq, const char* sid) {
    jintArray o = make(K_INTS, n_opts, 4);
    memcpy(o->data, opts, (size_t)n_opts * 4);
    jstring q = js(qseq), s = js(sid);
    const jlong c = NAT(open)(&g_env, NULL, device, o, het, q, s);
    drop(o); drop(q); drop(s);
    return c;
}
void h_close(int64_t ctx) { NAT(close)(&g_env, NULL, ctx); }
/* the message into buf (cap bytes) */
void h_last_error(int64_t ctx, char* buf, int cap) {
    jstring s = NAT(lastError)(&g_env, NULL, ctx);
    snprintf(buf, (size_t)cap, "%s", s ? (const char*)s->data : "");
    drop(s);
}
int h_load_fasta(int64_t ctx, const char* path) {
    jstring p = js(path);
    const int rc = NAT(loadFasta)(&g_env, NULL, ctx, p);
    drop(p);
    return rc;
}
int h_set_known_variants(int64_t ctx, const char* path) {
    jstring p = js(path);
    const int rc = NAT(setKnownVariants)(&g_env, NULL, ctx, p);
    drop(p);
    return rc;
}
int h_set_known_strs(int64_t ctx, const char* path) {
    jstring p = js(path);
    const int rc = NAT(setKnownSTRs)(&g_env, NULL, ctx, p);
    drop(p);
    return rc;
}
int h_call_bam(int64_t ctx, const char* bam, const char* out) {
    jstring b = js(bam), o = js(out);
    const int rc = NAT(callBam)(&g_env, NULL, ctx, b, o);
    drop(b); drop(o);
    return rc;
}
int h_call_region_bam(int64_t ctx, const char* bam, const char* seq, int64_t first, int64_t last, const char* out) {
    jstring b = js(bam), s = js(seq), o = js(out);
    const int rc = NAT(callRegionBam)(&g_env, NULL, ctx, b, s, first, last, o);
    drop(b); drop(s); drop(o);
    return rc;
}
int h_call_population_bams(int64_t ctx, const char* const* bams, int n, const char* out) {
    jobjectArray a = jstrings(bams, n);
    jstring o = js(out);
    const int rc = NAT(callPopulationBams)(&g_env, NULL, ctx, a, o);
    drop(a); drop(o);
    return rc;
}
int h_call_bam_multi(const int64_t* ctxs, int n, const char* bam, const char* out, int64_t window) {
    jlongArray c = jlongs(ctxs, n);
    jstring b = js(bam), o = js(out);
    const int rc = NAT(callBamMulti)(&g_env, NULL, c, b, o, window);
    drop(c); drop(b); drop(o);
    return rc;
}
int h_call_population_bams_multi(const int64_t* ctxs, int n, const char* const* bams, int nb, const char* out,
                                 int64_t window) {
    jlongArray c = jlongs(ctxs, n);
    jobjectArray a = jstrings(bams, nb);
    jstring o = js(out);
    const int rc = NAT(callPopulationBamsMulti)(&g_env, NULL, c, a, o, window);
    drop(c); drop(a); drop(o);
    return rc;
}
/* carvedRegions: the {seq, first, last} triples into out (3 per region), their number returned (-1 on error) */
int64_t h_carved_regions(int64_t ctx, int64_t* out, int64_t cap) {
    jobjectArray a = NAT(carvedRegions)(&g_env, NULL, ctx);
    if (!a) return -1;
    const jsize n = a->len;
    for (jsize i = 0; i < n && i < cap; i++) memcpy(out + 3 * i, ((jobject*)a->data)[i]->data, 3 * sizeof(int64_t));
    drop(a);
    return n;
}

/* processAlignments over a batch given as plain arrays (every array copied into a Java array first) */
static jintArray jints(const int32_t* v, int n) {
    jintArray a = make(K_INTS, n, 4);
    if (v) memcpy(a->data, v, (size_t)n * 4);
    return a;
}
static jbyteArray jbytes(const void* v, int64_t n) {
    jbyteArray a = make(K_BYTES, (jsize)n, 1);
    if (v) memcpy(a->data, v, (size_t)n);
    return a;
}
int h_process_alignments(int64_t ctx, int n, const int32_t* seq_id, const int32_t* first, const int32_t* flags,
                         const int32_t* rg, const int64_t* cig_off, const int32_t* cig_n, const int32_t* cig, int n_cig,
                         const int64_t* seq_off, const int32_t* seq_len, const char* bases, const char* quals, int64_t n_bases,
                         const uint8_t* has_q) {
    jintArray a0 = jints(seq_id, n), a1 = jints(first, n), a2 = jints(flags, n), a3 = jints(rg, n);
    jlongArray a4 = jlongs(cig_off, n);
    jintArray a5 = jints(cig_n, n), a6 = jints(cig, n_cig);
    jlongArray a7 = jlongs(seq_off, n);
    jintArray a8 = jints(seq_len, n);
    jbyteArray a9 = jbytes(bases, n_bases), a10 = jbytes(quals, n_bases), a11 = jbytes(has_q, n);
    const int rc = NAT(processAlignments)(&g_env, NULL, ctx, a0, a1, a2, a3, a4, a5, a6, a7, a8, a9, a10, a11);
    drop(a0); drop(a1); drop(a2); drop(a3); drop(a4); drop(a5); drop(a6); drop(a7); drop(a8); drop(a9); drop(a10); drop(a11);
    return rc;
}
int h_notify_end(int64_t ctx) { return NAT(notifyEnd)(&g_env, NULL, ctx); }
/* fetchSites: the records' bytes into out (cap bytes); their byte count (-1: null returned); *le = the buffer's order
   was set to LITTLE_ENDIAN */
int64_t h_fetch_sites(int64_t ctx, void* out, int64_t cap, int* le) {
    g_order_le = 0;
    jobject b = NAT(fetchSites)(&g_env, NULL, ctx);
    *le = g_order_le;
    if (!b) return -1;
    const int64_t n = b->len;
    memcpy(out, b->data, (size_t)(n < cap ? n : cap));
    drop(b);
    return n;
}
