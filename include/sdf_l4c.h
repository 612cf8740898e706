/* sdf_l4c.h -- drop-in replacement for the L4CasADi-generated library libsdf_l4c.so.
 *
 * acados links the CasADi-generated constraint functions of the OCP
 * (quad_rollpitchyawrate_sdf_constr_h_fun_jac_uxt_zt, ..._constr_h_e_..., and the cost functions
 * when flags.sdf_cost) against `sdf_l4c` found in solver_options.model_external_shared_lib_dir
 * (sdf_nmpc/ocp.py:100-102); the library is produced by
 *     l4casadi.L4CasADi(sdf, model_expects_batch_dim=True, build_dir=cache/codegen/<name>,
 *                       name='sdf_l4c', device=..., with_jacobian=True, with_hessian=False)
 * (sdf_nmpc/gen_model.py:38-39) and called as sdf_l4c(vertcat(Co_p_B, latent)) (gen_model.py:60).
 * Nmpc.eval reaches the same symbols through CasADi's external() (model/base_model.py:119-125).
 *
 * These are the CasADi external-function C ABI entry points such a library exports
 * (casadi_real = double, casadi_int = long long).  L4CasADi 1.4.1's exact emitted symbol set is not
 * verifiable in this environment (the package is not installed); this set is the CasADi external
 * protocol for a 1-in/1-out function with a Jacobian ("jac_" + name: inputs = nominal inputs followed
 * by nominal outputs, output = dense d out / d in) and a first-order adjoint ("adj1_" + name).
 *
 * Weights: an .sdfw file at $SDFNMPC_WEIGHTS, else "sdf_l4c.sdfw" next to the loaded library.
 * Device: $SDFNMPC_DEVICE (default 0).  Errors return non-zero (acados -> solver status ->
 * Nmpc.solve fail_count, controller.py:72-81); nothing throws across the ABI.
 */
#ifndef SDF_L4C_H
#define SDF_L4C_H

#ifdef __cplusplus
extern "C" {
#endif

typedef double sdf_l4c_real;
typedef long long sdf_l4c_int;

/* f: [Co_p_B(3); latent(L)] ((3 + L) x 1) -> df (1 x 1); L = the loaded network's size_latent (128 for
 * the deployed net, gen_model.py:39,60 / network/neural_df.py:16; any L <= 1024).  The sparsity queries
 * load the network first, so the patterns carry its width. */
int sdf_l4c(const sdf_l4c_real** arg, sdf_l4c_real** res, sdf_l4c_int* iw, sdf_l4c_real* w, int mem);
sdf_l4c_int sdf_l4c_n_in(void);
sdf_l4c_int sdf_l4c_n_out(void);
const sdf_l4c_int* sdf_l4c_sparsity_in(sdf_l4c_int i);
const sdf_l4c_int* sdf_l4c_sparsity_out(sdf_l4c_int i);
int sdf_l4c_work(sdf_l4c_int* sz_arg, sdf_l4c_int* sz_res, sdf_l4c_int* sz_iw, sdf_l4c_int* sz_w);
const char* sdf_l4c_name_in(sdf_l4c_int i);
const char* sdf_l4c_name_out(sdf_l4c_int i);
int sdf_l4c_checkout(void);
void sdf_l4c_release(int mem);
void sdf_l4c_incref(void);
void sdf_l4c_decref(void);

/* Jacobian: (in ((3+L)x1), out (1x1)) -> d out / d in (1 x (3+L), dense) */
int jac_sdf_l4c(const sdf_l4c_real** arg, sdf_l4c_real** res, sdf_l4c_int* iw, sdf_l4c_real* w, int mem);
sdf_l4c_int jac_sdf_l4c_n_in(void);
sdf_l4c_int jac_sdf_l4c_n_out(void);
const sdf_l4c_int* jac_sdf_l4c_sparsity_in(sdf_l4c_int i);
const sdf_l4c_int* jac_sdf_l4c_sparsity_out(sdf_l4c_int i);
int jac_sdf_l4c_work(sdf_l4c_int* sz_arg, sdf_l4c_int* sz_res, sdf_l4c_int* sz_iw, sdf_l4c_int* sz_w);

/* Adjoint: (in ((3+L)x1), out (1x1), adj_out (1x1)) -> adj_out * d out / d in ((3+L) x 1) */
int adj1_sdf_l4c(const sdf_l4c_real** arg, sdf_l4c_real** res, sdf_l4c_int* iw, sdf_l4c_real* w, int mem);
sdf_l4c_int adj1_sdf_l4c_n_in(void);
sdf_l4c_int adj1_sdf_l4c_n_out(void);
const sdf_l4c_int* adj1_sdf_l4c_sparsity_in(sdf_l4c_int i);
const sdf_l4c_int* adj1_sdf_l4c_sparsity_out(sdf_l4c_int i);
int adj1_sdf_l4c_work(sdf_l4c_int* sz_arg, sdf_l4c_int* sz_res, sdf_l4c_int* sz_iw, sdf_l4c_int* sz_w);

/* out-of-band configuration (not part of the CasADi protocol): load weights / select device
 * explicitly instead of the environment; returns 0 on success. */
int sdf_l4c_configure(const char* weights_path, int device);
const char* sdf_l4c_last_error(void);

#ifdef __cplusplus
}
#endif
#endif /* SDF_L4C_H */
