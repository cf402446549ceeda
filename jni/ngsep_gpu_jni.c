/*
 * ngsep_gpu_jni.c -- the JNI binding a NGSEPcore maintainer adds for ngsep.discovery.gpu.GpuPileupEngine
 * (INTEGRATION.md section 2 holds the Java class).  Every native forwards to one entry point of include/ngsep_gpu.h;
 * strings are UTF-8 copies, arrays are taken with Get<Type>ArrayElements around the call (released with JNI_ABORT;
 * critical sections only around short copies), errors come back as the int status the Java side turns into an IOException with
 * ngsep_last_error.  Build (with a JDK):
 *   gcc -O2 -shared -fPIC -I$JAVA_HOME/include -I$JAVA_HOME/include/linux -Iinclude jni/ngsep_gpu_jni.c \
 *       -Lngsepcore_amd/lib -lngsep_amd -Wl,-rpath,'$ORIGIN' -o libngsep_amd_jni.so
 * tests/test_jni_shim.py compiles this file against tests/jni_harness (a JNIEnv of its own, the image has no JDK) and
 * drives the natives the way the JVM would.
 */
#include <jni.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include "ngsep_gpu.h"

#define CTX(p) ((ngsep_ctx*)(intptr_t)(p))
#define FN(name) JNICALL Java_ngsep_discovery_gpu_GpuPileupEngine_##name

/* a UTF-8 copy of a Java string (NULL for null), released by utf_free */
typedef struct { jstring s; const char* c; } utf;
static utf utf_get(JNIEnv* env, jstring s) {
    utf u = {s, NULL};
    if (s) u.c = (*env)->GetStringUTFChars(env, s, NULL);
    return u;
}
static void utf_free(JNIEnv* env, utf u) {
    if (u.s && u.c) (*env)->ReleaseStringUTFChars(env, u.s, u.c);
}
static void throw_io(JNIEnv* env, const char* msg) {
    jclass ex = (*env)->FindClass(env, "java/io/IOException");
    if (ex) (*env)->ThrowNew(env, ex, msg);
}

/* options: ngsep_params fields in the order GpuPileupEngine.optionArray() writes them */
static void params_from(JNIEnv* env, jintArray opts, jdouble h, ngsep_params* p) {
    ngsep_params_default(p);
    const jsize n = opts ? (*env)->GetArrayLength(env, opts) : 0;
    jint* o = opts ? (*env)->GetIntArrayElements(env, opts, NULL) : NULL;
    int32_t* f[] = {&p->min_mq, &p->max_alns_per_start, &p->ignore5, &p->ignore3, &p->max_base_qs, &p->min_quality, &p->ploidy,
                    &p->process_nonunique, &p->process_secondary, &p->ignore_lowercase_ref, &p->call_embedded,
                    &p->calc_strand_bias, &p->print_sample_ploidy, &p->het_rate_set, &p->query_first, &p->query_last,
                    &p->multisample, &p->coverage_stats, &p->max_coverage, &p->relative_allele_counts, &p->rac_min_rd,
                    &p->rac_min_bq, &p->indel_passthrough};
    for (jsize i = 0; i < n && i < (jsize)(sizeof f / sizeof f[0]); i++) *f[i] = o[i];
    if (o) (*env)->ReleaseIntArrayElements(env, opts, o, JNI_ABORT);
    p->het_rate = h;
}

JNIEXPORT jlong FN(open)(JNIEnv* env, jclass k, jint dev, jintArray opts, jdouble h, jstring qseq, jstring sid) {
    (void)k;
    ngsep_params p;
    params_from(env, opts, h, &p);
    utf q = utf_get(env, qseq), s = utf_get(env, sid);
    if (q.c) strncpy(p.query_seq, q.c, sizeof p.query_seq - 1);
    if (s.c) strncpy(p.sample_id, s.c, sizeof p.sample_id - 1);
    utf_free(env, q);
    utf_free(env, s);
    ngsep_ctx* c = NULL;
    const int rc = ngsep_open(dev, &p, &c);
    if (rc != NGSEP_OK) {
        throw_io(env, c ? ngsep_last_error(c) : "ngsep_open failed");
        if (c) ngsep_close(c);
        return 0;
    }
    return (jlong)(intptr_t)c;
}

JNIEXPORT void FN(close)(JNIEnv* env, jclass k, jlong ctx) {
    (void)env; (void)k;
    if (ctx) ngsep_close(CTX(ctx));
}

JNIEXPORT jstring FN(lastError)(JNIEnv* env, jclass k, jlong ctx) {
    (void)k;
    return (*env)->NewStringUTF(env, ctx ? ngsep_last_error(CTX(ctx)) : "no context");
}

/* ReferenceGenome(filename) */
JNIEXPORT jint FN(loadFasta)(JNIEnv* env, jclass k, jlong ctx, jstring path) {
    (void)k;
    utf u = utf_get(env, path);
    const int rc = ngsep_load_fasta(CTX(ctx), u.c);
    utf_free(env, u);
    return rc;
}

/* SingleSampleVariantsDetector.findSNVS on a BAM (:896-931) */
JNIEXPORT jint FN(callBam)(JNIEnv* env, jclass k, jlong ctx, jstring bam, jstring out) {
    (void)k;
    utf b = utf_get(env, bam), o = utf_get(env, out);
    const int rc = ngsep_call_bam(CTX(ctx), b.c, o.c);
    utf_free(env, b);
    utf_free(env, o);
    return rc;
}

/* findSNVS with -querySeq seq -first first -last last (AlignmentsPileupGenerator.java:242-254) */
JNIEXPORT jint FN(callRegionBam)(JNIEnv* env, jclass k, jlong ctx, jstring bam, jstring seq, jlong first, jlong last,
                                 jstring out) {
    (void)k;
    utf b = utf_get(env, bam), s = utf_get(env, seq), o = utf_get(env, out);
    const int rc = ngsep_call_region_bam(CTX(ctx), b.c, s.c, first, last, o.c);
    utf_free(env, b);
    utf_free(env, s);
    utf_free(env, o);
    return rc;
}

/* the strings of a String[] as UTF-8 copies (released by strings_free) */
static const char** strings_get(JNIEnv* env, jobjectArray arr, jsize* n_out) {
    const jsize n = arr ? (*env)->GetArrayLength(env, arr) : 0;
    const char** v = (const char**)calloc((size_t)(n > 0 ? n : 1), sizeof(char*));
    for (jsize i = 0; i < n; i++) {
        jstring s = (jstring)(*env)->GetObjectArrayElement(env, arr, i);
        v[i] = s ? (*env)->GetStringUTFChars(env, s, NULL) : NULL;
    }
    *n_out = n;
    return v;
}
static void strings_free(JNIEnv* env, jobjectArray arr, const char** v, jsize n) {
    for (jsize i = 0; i < n; i++) {
        jstring s = (jstring)(*env)->GetObjectArrayElement(env, arr, i);
        if (s && v[i]) (*env)->ReleaseStringUTFChars(env, s, v[i]);
    }
    free((void*)v);
}

/* MultisampleVariantsDetector.run on BAM files (:421-459) */
JNIEXPORT jint FN(callPopulationBams)(JNIEnv* env, jclass k, jlong ctx, jobjectArray bams, jstring out) {
    (void)k;
    jsize n = 0;
    const char** b = strings_get(env, bams, &n);
    utf o = utf_get(env, out);
    const int rc = ngsep_call_population_bams(CTX(ctx), b, (int32_t)n, o.c);
    utf_free(env, o);
    strings_free(env, bams, b, n);
    return rc;
}

/* several devices of this process (ABI 11): contexts[k] one per device, windows from one queue */
JNIEXPORT jint FN(callBamMulti)(JNIEnv* env, jclass k, jlongArray contexts, jstring bam, jstring out, jlong window) {
    (void)k;
    const jsize n = (*env)->GetArrayLength(env, contexts);
    jlong* c = (*env)->GetLongArrayElements(env, contexts, NULL);
    ngsep_ctx** v = (ngsep_ctx**)calloc((size_t)(n > 0 ? n : 1), sizeof(ngsep_ctx*));
    for (jsize i = 0; i < n; i++) v[i] = CTX(c[i]);
    (*env)->ReleaseLongArrayElements(env, contexts, c, JNI_ABORT);
    utf b = utf_get(env, bam), o = utf_get(env, out);
    const int rc = ngsep_call_bam_multi(v, (int32_t)n, b.c, o.c, window);
    utf_free(env, b);
    utf_free(env, o);
    free(v);
    return rc;
}

JNIEXPORT jint FN(callPopulationBamsMulti)(JNIEnv* env, jclass k, jlongArray contexts, jobjectArray bams, jstring out,
                                           jlong window) {
    (void)k;
    const jsize n = (*env)->GetArrayLength(env, contexts);
    jlong* c = (*env)->GetLongArrayElements(env, contexts, NULL);
    ngsep_ctx** v = (ngsep_ctx**)calloc((size_t)(n > 0 ? n : 1), sizeof(ngsep_ctx*));
    for (jsize i = 0; i < n; i++) v[i] = CTX(c[i]);
    (*env)->ReleaseLongArrayElements(env, contexts, c, JNI_ABORT);
    jsize nb = 0;
    const char** b = strings_get(env, bams, &nb);
    utf o = utf_get(env, out);
    const int rc = ngsep_call_population_bams_multi(v, (int32_t)n, b, (int32_t)nb, o.c, window);
    utf_free(env, o);
    strings_free(env, bams, b, nb);
    free(v);
    return rc;
}

/* path A: one batch of filtered, coordinate-sorted alignments (AlignmentsPileupGenerator.processAlignment).  The call
 * projects the batch on every host thread and can wait on the device, far too long to hold critical sections (a JVM's
 * GC would stall behind them): the arrays are taken with Get<Type>ArrayElements (a copy or a pin the GC can live with)
 * and released with JNI_ABORT (nothing is written back).  A null element pointer (the JVM out of memory) throws
 * OutOfMemoryError and returns NGSEP_E_INVALID. */
JNIEXPORT jint FN(processAlignments)(JNIEnv* env, jclass k, jlong ctx, jintArray seqId, jintArray first, jintArray flags,
                                     jintArray rg, jlongArray cigOff, jintArray cigN, jintArray cig, jlongArray seqOff,
                                     jintArray seqLen, jbyteArray bases, jbyteArray quals, jbyteArray hasQ) {
    (void)k;
    jintArray ia[] = {seqId, first, flags, rg, cigN, cig, seqLen};
    jint* ie[7] = {NULL};
    jlongArray la[] = {cigOff, seqOff};
    jlong* le[2] = {NULL};
    jbyteArray ba[] = {bases, quals, hasQ};
    jbyte* be[3] = {NULL};
    int ok = 1;
    for (int i = 0; i < 7 && ok; i++) ok = (ie[i] = (*env)->GetIntArrayElements(env, ia[i], NULL)) != NULL;
    for (int i = 0; i < 2 && ok; i++) ok = (le[i] = (*env)->GetLongArrayElements(env, la[i], NULL)) != NULL;
    for (int i = 0; i < 3 && ok; i++) ok = !ba[i] || (be[i] = (*env)->GetByteArrayElements(env, ba[i], NULL)) != NULL;
    int rc = NGSEP_E_INVALID;
    if (ok) {
        ngsep_read_batch b;
        b.n_reads = (*env)->GetArrayLength(env, first);
        b.seq_id = (const int32_t*)ie[0];
        b.first = (const int32_t*)ie[1];
        b.flags = (const int32_t*)ie[2];
        b.read_group = (const int32_t*)ie[3];
        b.cigar_off = (const int64_t*)le[0];
        b.cigar_n = (const int32_t*)ie[4];
        b.cigar = (const int32_t*)ie[5];
        b.seq_off = (const int64_t*)le[1];
        b.seq_len = (const int32_t*)ie[6];
        b.bases = (const char*)be[0];
        b.quals = (const char*)be[1];
        b.has_quals = (const uint8_t*)be[2];
        rc = ngsep_process_alignments(CTX(ctx), &b);
    } else {
        jclass oom = (*env)->FindClass(env, "java/lang/OutOfMemoryError");
        if (oom) (*env)->ThrowNew(env, oom, "processAlignments: array elements could not be obtained");
    }
    for (int i = 0; i < 3; i++) if (be[i]) (*env)->ReleaseByteArrayElements(env, ba[i], be[i], JNI_ABORT);
    for (int i = 0; i < 2; i++) if (le[i]) (*env)->ReleaseLongArrayElements(env, la[i], le[i], JNI_ABORT);
    for (int i = 0; i < 7; i++) if (ie[i]) (*env)->ReleaseIntArrayElements(env, ia[i], ie[i], JNI_ABORT);
    return rc;
}

/* AlignmentsPileupGenerator.notifyEndOfAlignments */
JNIEXPORT jint FN(notifyEnd)(JNIEnv* env, jclass k, jlong ctx) {
    (void)env; (void)k;
    return ngsep_notify_end(CTX(ctx));
}

/* the called sites as packed ngsep_site_out records (152 B each) in a heap ByteBuffer whose order is set to
 * ByteOrder.LITTLE_ENDIAN (the records' own; a wrapped buffer defaults to BIG_ENDIAN, which would byte-swap every
 * getInt / getLong).  A failing fetch throws IOException (the method's declared exception) and returns null. */
JNIEXPORT jobject FN(fetchSites)(JNIEnv* env, jclass k, jlong ctx) {
    (void)k;
    int64_t n = 0;
    if (ngsep_fetch_sites(CTX(ctx), NULL, 0, &n) != NGSEP_OK) {
        throw_io(env, ngsep_last_error(CTX(ctx)));
        return NULL;
    }
    ngsep_site_out* buf = (ngsep_site_out*)malloc((size_t)(n > 0 ? n : 1) * sizeof(ngsep_site_out));
    if (!buf) {
        throw_io(env, "fetchSites: out of host memory");
        return NULL;
    }
    if (ngsep_fetch_sites(CTX(ctx), buf, n, &n) != NGSEP_OK) {
        free(buf);
        throw_io(env, ngsep_last_error(CTX(ctx)));
        return NULL;
    }
    ngsep_clear_sites(CTX(ctx));
    const jsize bytes = (jsize)(n * (int64_t)sizeof(ngsep_site_out));
    jbyteArray arr = (*env)->NewByteArray(env, bytes);
    if (arr) (*env)->SetByteArrayRegion(env, arr, 0, bytes, (const jbyte*)buf);
    free(buf);
    if (!arr) return NULL;                             /* (NewByteArray has thrown OutOfMemoryError) */
    jclass bb = (*env)->FindClass(env, "java/nio/ByteBuffer");
    jmethodID wrap = (*env)->GetStaticMethodID(env, bb, "wrap", "([B)Ljava/nio/ByteBuffer;");
    jobject buffer = (*env)->CallStaticObjectMethod(env, bb, wrap, arr);
    if (!buffer) return NULL;
    jclass bo = (*env)->FindClass(env, "java/nio/ByteOrder");
    jfieldID lef = (*env)->GetStaticFieldID(env, bo, "LITTLE_ENDIAN", "Ljava/nio/ByteOrder;");
    jobject le = (*env)->GetStaticObjectField(env, bo, lef);
    jmethodID order = (*env)->GetMethodID(env, bb, "order", "(Ljava/nio/ByteOrder;)Ljava/nio/ByteBuffer;");
    return (*env)->CallObjectMethod(env, buffer, order, le);
}

/* the VCF text of fetched record i (indel / STR records, ABI 6) */
JNIEXPORT jstring FN(siteLine)(JNIEnv* env, jclass k, jlong ctx, jlong i) {
    (void)k;
    char buf[4096];
    const int64_t n = ngsep_site_vcf_line(CTX(ctx), i, buf, sizeof buf);
    if (n < 0) return NULL;
    if (n < (int64_t)sizeof buf) return (*env)->NewStringUTF(env, buf);
    char* big = (char*)malloc((size_t)n + 1);
    if (!big) return NULL;
    ngsep_site_vcf_line(CTX(ctx), i, big, n + 1);
    jstring s = (*env)->NewStringUTF(env, big);
    free(big);
    return s;
}

/* -knownVariants (SingleSampleVariantsDetector.findSNVS :896-906) and -knownSTRs (:906-912) */
JNIEXPORT jint FN(setKnownVariants)(JNIEnv* env, jclass k, jlong ctx, jstring vcf) {
    (void)k;
    utf u = utf_get(env, vcf);
    const int rc = ngsep_set_known_variants(CTX(ctx), u.c);
    utf_free(env, u);
    return rc;
}
JNIEXPORT jint FN(setKnownSTRs)(JNIEnv* env, jclass k, jlong ctx, jstring path) {
    (void)k;
    utf u = utf_get(env, path);
    const int rc = ngsep_set_known_strs(CTX(ctx), u.c);
    utf_free(env, u);
    return rc;
}

/* pass-through mode: the regions left to the caller's indel path, {sequence index, first, last} (1-based) */
JNIEXPORT jobjectArray FN(carvedRegions)(JNIEnv* env, jclass k, jlong ctx) {
    (void)k;
    int64_t n = 0;
    if (ngsep_fetch_carved_regions(CTX(ctx), NULL, NULL, NULL, 0, &n) != NGSEP_OK) return NULL;
    int32_t* seq = (int32_t*)malloc((size_t)(n ? n : 1) * sizeof(int32_t));
    int64_t* first = (int64_t*)malloc((size_t)(n ? n : 1) * sizeof(int64_t));
    int64_t* last = (int64_t*)malloc((size_t)(n ? n : 1) * sizeof(int64_t));
    if (!seq || !first || !last) { free(seq); free(first); free(last); return NULL; }
    ngsep_fetch_carved_regions(CTX(ctx), seq, first, last, n, &n);
    jobjectArray out = (*env)->NewObjectArray(env, (jsize)n, (*env)->FindClass(env, "[J"), NULL);
    for (int64_t i = 0; out && i < n; i++) {
        const jlong v[3] = {seq[i], first[i], last[i]};
        jlongArray a = (*env)->NewLongArray(env, 3);
        (*env)->SetLongArrayRegion(env, a, 0, 3, v);
        (*env)->SetObjectArrayElement(env, out, (jsize)i, a);
    }
    free(seq);
    free(first);
    free(last);
    ngsep_clear_carved_regions(CTX(ctx));
    return out;
}

/* CoverageStatisticsCalculator.processFile (:99-122) and its counts */
JNIEXPORT jint FN(coverageBam)(JNIEnv* env, jclass k, jlong ctx, jstring bam, jstring out) {
    (void)k;
    utf b = utf_get(env, bam), o = utf_get(env, out);
    const int rc = ngsep_coverage_bam(CTX(ctx), b.c, o.c ? o.c : "-");
    utf_free(env, b);
    utf_free(env, o);
    return rc;
}
JNIEXPORT jint FN(fetchCoverage)(JNIEnv* env, jclass k, jlong ctx, jlongArray counts, jlongArray unique, jlongArray more) {
    (void)k;
    jlong* c = (jlong*)(*env)->GetPrimitiveArrayCritical(env, counts, NULL);
    jlong* u = (jlong*)(*env)->GetPrimitiveArrayCritical(env, unique, NULL);
    jlong* m = (jlong*)(*env)->GetPrimitiveArrayCritical(env, more, NULL);
    /* (a short copy of the histograms: critical sections are fine here) */
    const int rc = c && u && m ? ngsep_fetch_coverage(CTX(ctx), (int64_t*)c, (int64_t*)u, (int64_t*)&m[0], (int64_t*)&m[1])
                               : NGSEP_E_INVALID;
    if (m) (*env)->ReleasePrimitiveArrayCritical(env, more, m, 0);
    if (u) (*env)->ReleasePrimitiveArrayCritical(env, unique, u, 0);
    if (c) (*env)->ReleasePrimitiveArrayCritical(env, counts, c, 0);
    return rc;
}

/* RelativeAlleleCountsCalculator (:183-331): the report, then its distributions for the getters */
JNIEXPORT jint FN(racBam)(JNIEnv* env, jclass k, jlong ctx, jstring bam, jstring out) {
    (void)k;
    utf b = utf_get(env, bam), o = utf_get(env, out);
    const int rc = ngsep_rac_bam(CTX(ctx), b.c, o.c ? o.c : "-");
    utf_free(env, b);
    utf_free(env, o);
    return rc;
}
JNIEXPORT jint FN(fetchRac)(JNIEnv* env, jclass k, jlong ctx, jdoubleArray prop, jdoubleArray nAlleles, jdoubleArray moments) {
    (void)k;
    double* p = (double*)(*env)->GetPrimitiveArrayCritical(env, prop, NULL);
    double* a = (double*)(*env)->GetPrimitiveArrayCritical(env, nAlleles, NULL);
    double* m = (double*)(*env)->GetPrimitiveArrayCritical(env, moments, NULL);
    const int rc = p && a && m ? ngsep_fetch_rac(CTX(ctx), p, a, m) : NGSEP_E_INVALID;
    if (m) (*env)->ReleasePrimitiveArrayCritical(env, moments, m, 0);
    if (a) (*env)->ReleasePrimitiveArrayCritical(env, nAlleles, a, 0);
    if (p) (*env)->ReleasePrimitiveArrayCritical(env, prop, p, 0);
    return rc;
}
