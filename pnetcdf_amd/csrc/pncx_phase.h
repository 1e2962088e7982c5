/*
 * pncx_phase.h -- per-phase timing of the host-buffer paths (internal to
 * libpncx.so; the public switch is pncx_phases() in include/pncx.h).
 *
 *   double t = PH_T0();  ...  PH_ADD(PH_PUT_WRITE, t);
 *
 * PH_T0() is 0 when recording is off, and PH_ADD then does nothing, so the
 * cost on the product path is one load and one branch.
 */
#ifndef PNCX_PHASE_H
#define PNCX_PHASE_H

enum {
    PH_PUT_PLAN,        /* checks, request plan, file runs                 */
    PH_PUT_REGISTER,    /* pinning the user buffer for the call            */
    PH_PUT_CONVERT,     /* the conversion call(s), enqueue to data ready   */
    PH_PUT_WRITE,       /* submitting + writing the file runs              */
    PH_PUT_WAIT,        /* waiting for the I/O pool at the end             */
    PH_PUT_UNREGISTER,
    PH_PUT_TOTAL,
    PH_GET_PLAN,
    PH_GET_REGISTER,
    PH_GET_READ,        /* reads submitted + waited for                    */
    PH_GET_CONVERT,
    PH_GET_UNREGISTER,
    PH_GET_TOTAL,
    PH_CONV_LOCK,       /* host_staged: context lock + pin checks          */
    PH_CONV_ENQUEUE,    /* H2D / kernel / D2H enqueue calls                */
    PH_CONV_SYNC,       /* stream synchronisation                          */
    PH_CONV_STATUS,     /* status words back                               */
    PH_CONV_UNPIN,
    PH_GPU_H2D,         /* HIP-event intervals on the device               */
    PH_GPU_KERNEL,
    PH_GPU_D2H,
    PH_WIN_MAP,         /* a file window mapped and registered             */
    PH_WIN_USE,         /* a request converted through a file window       */
    PH_PUT_GROW,        /* appended pages allocated while the GPU converts */
    PH_WARM,            /* the create/open warm-up thread, start to end    */
    PH_PRELOAD,         /* enddef: code objects of the defined types        */
    PH_N
};

#ifdef __cplusplus
extern "C" {
#endif
extern int pncx_ph_on;
double pncx_ph_now(void);
void pncx_ph_add_us(int id, double us);
#ifdef __cplusplus
}
#endif

#define PH_T0() (pncx_ph_on ? pncx_ph_now() : 0.0)
#define PH_ADD(id, t0) do { if (pncx_ph_on && (t0) > 0.0) pncx_ph_add_us((id), pncx_ph_now() - (t0)); } while (0)

#endif
