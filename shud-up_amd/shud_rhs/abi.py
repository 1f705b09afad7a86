"""ctypes mirror of include/shud_rhs.h (the C-ABI boundary).

Struct layouts here must match the header field for field; tests/test_abi.py checks sizes and that
libshud_rhs.so exports every function the header declares.
"""
import ctypes as C

c_int32_p = C.POINTER(C.c_int32)
c_double_p = C.POINTER(C.c_double)

SHUD_OK = 0
SHUD_ERR_PHYSICS = -1
SHUD_ERR_ARG = -2
SHUD_ERR_HIP = -3
SHUD_ERR_NCCL = -4
SHUD_ERR_UNSUPPORTED = -5

SHUD_MODE_SERIAL = 0
SHUD_MODE_OMP = 1
SHUD_WHERE_HOST = 0
SHUD_WHERE_DEVICE = 1

EF_NAN_QELE = 0x01
EF_EFFKH = 0x02
EF_ET_NEG = 0x04
EF_ET_NAN = 0x08
EF_AET_WARN = 0x10
EF_ET_RA = 0x20
EF_ET_PT_NAN = 0x40
SHUD_TSR_OFF, SHUD_TSR_NO_TIME, SHUD_TSR_CACHED, SHUD_TSR_RECOMPUTE = 0, 1, 2, 3

MESH_FIELDS = [
    ("num_ele", C.c_int32), ("num_riv", C.c_int32), ("num_seg", C.c_int32), ("close_boundary", C.c_int32),
    ("nabr", c_int32_p), ("area", c_double_p), ("z_surf", c_double_p), ("z_bottom", c_double_p),
    ("depression", c_double_p), ("edge", c_double_p), ("dist2nabor", c_double_p), ("dist2edge", c_double_p),
    ("avg_rough", c_double_p), ("rough", c_double_p), ("ibc", c_int32_p), ("iss", c_int32_p), ("ilake", c_int32_p),
    ("riv_down", c_int32_p), ("riv_bc", c_int32_p), ("riv_length", c_double_p), ("riv_bed_slope", c_double_p),
    ("riv_dist2down", c_double_p), ("riv_avg_rough", c_double_p), ("riv_depth", c_double_p),
    ("riv_bottom_width", c_double_p), ("riv_bankslope", c_double_p), ("riv_ksath", c_double_p),
    ("riv_bedthick", c_double_p),
    ("seg_ele", c_int32_p), ("seg_riv", c_int32_p), ("seg_length", c_double_p), ("seg_cwr", c_double_p),
    ("num_lake", C.c_int32), ("lake_bathy_off", c_int32_p), ("lake_bathy_y", c_double_p),
    ("lake_bathy_a", c_double_p),
]
PARAM_NAMES = ["aquifer_depth", "macD", "macKsatH", "geo_vAreaF", "KsatH", "KsatV", "infKsatV", "hAreaF",
               "macKsatV", "ThetaS", "ThetaR", "Beta", "infD", "Sy", "RzD", "VegFrac", "ImpAF"]
STEP_ARRAYS = ["net_prep", "pot_evap", "pot_tran", "etp", "lai", "fu_surf", "fu_sub", "e_ic", "u_satn",
               "ugw_stale"]
DIAG_ELE3 = ["qele_surf", "qele_sub"]
DIAG_ELE = ["qele_surf_tot", "qele_sub_tot", "q_infil", "q_exfil", "q_recharge", "q_es", "q_eu", "q_eg",
            "q_tu", "q_tg", "q_eta", "e_ic", "u_satn", "i_beta", "eff_kh", "qe2r_surf", "qe2r_sub"]
DIAG_SEG = ["qseg_surf", "qseg_sub"]
DIAG_RIV = ["qriv_down", "qriv_up", "qriv_surf", "qriv_sub"]
DIAG_LAKE = ["q_lake_surf", "q_lake_sub", "q_lake_rivin", "q_lake_evap", "q_lake_prcp", "lake_toparea"]


class ShudMeshSoA(C.Structure):
    _fields_ = MESH_FIELDS


class ShudParamsSoA(C.Structure):
    _fields_ = [(n, c_double_p) for n in PARAM_NAMES]


class ShudStepInputs(C.Structure):
    _fields_ = [(n, c_double_p) for n in STEP_ARRAYS] + [
        ("ele_ybc", c_double_p), ("n_ele_ybc", C.c_int32),
        ("ele_qbc", c_double_p), ("n_ele_qbc", C.c_int32),
        ("riv_ybc", c_double_p), ("n_riv_ybc", C.c_int32),
        ("riv_qbc", c_double_p), ("n_riv_qbc", C.c_int32),
        ("prcp", c_double_p),
    ]


class ShudRhsOptions(C.Structure):
    _fields_ = [("mode", C.c_int32), ("device", C.c_int32), ("stream", C.c_void_p), ("check_errors", C.c_int32)]


class ShudFluxOut(C.Structure):
    _fields_ = [(n, c_double_p) for n in DIAG_ELE3[:2] + DIAG_ELE[:2] + ["q_infil", "q_exfil", "q_recharge",
                                                                        "q_es", "q_eu", "q_eg", "q_tu", "q_tg",
                                                                        "q_eta", "e_ic", "u_satn", "i_beta",
                                                                        "eff_kh", "qe2r_surf", "qe2r_sub",
                                                                        "qseg_surf", "qseg_sub", "qriv_down",
                                                                        "qriv_up", "qriv_surf", "qriv_sub"]
                                                                      + DIAG_LAKE]


FLUXOUT_ORDER = [f[0] for f in ShudFluxOut._fields_]


class ShudErr(C.Structure):
    _fields_ = [("flags", C.c_uint32), ("exit_code", C.c_int32), ("first_index", C.c_int32 * 8),
                ("n_aet_warn", C.c_int64), ("message", C.c_char * 256)]


class ShudPartition(C.Structure):
    _fields_ = [("rank", C.c_int32), ("nranks", C.c_int32), ("n_own_ele", C.c_int32),
                ("n_segghost_ele", C.c_int32), ("n_own_riv", C.c_int32),
                ("ele_send_off", c_int32_p), ("ele_send_idx", c_int32_p), ("ele_recv_off", c_int32_p),
                ("riv_send_off", c_int32_p), ("riv_send_idx", c_int32_p), ("riv_recv_off", c_int32_p),
                ("ele_gid", c_int32_p), ("riv_gid", c_int32_p), ("nccl_unique_id", C.c_char_p)]


# ---- include/shud_et.h (ET-step prelude) ----
class ShudEtMeshSoA(C.Structure):
    _fields_ = [("num_ele", C.c_int32), ("iforc", c_int32_p), ("ilc", c_int32_p), ("imf", c_int32_p),
                ("z_surf", c_double_p), ("albedo", c_double_p), ("fix_pressure", c_double_p), ("wind_h", c_double_p),
                ("veg_frac", c_double_p), ("ilake", c_int32_p), ("nx", c_double_p), ("ny", c_double_p),
                ("nz", c_double_p)]


ET_PARAM_D = ["cPrep", "cTemp", "cLAItsd", "cMF", "cETP", "cISmax"]


class ShudEtParams(C.Structure):
    _fields_ = [(n, C.c_double) for n in ET_PARAM_D] + [
        ("radiation_input_mode", C.c_int32), ("terrain_radiation", C.c_int32), ("rad_factor_cap", C.c_double),
        ("rad_cosz_min", C.c_double), ("cryosphere", C.c_int32), ("ft_surf_day", C.c_int32),
        ("ft_sub_day", C.c_int32), ("ft_surf_max", C.c_double), ("ft_surf_min", C.c_double),
        ("ft_sub_max", C.c_double), ("ft_sub_min", C.c_double)]


class ShudEtForcing(C.Structure):
    _fields_ = [("t", C.c_double), ("t_next", C.c_double), ("n_station", C.c_int32), ("station", c_double_p),
                ("station_z", c_double_p), ("n_lai_col", C.c_int32), ("lai_row", c_double_p),
                ("n_mf_col", C.c_int32), ("mf_row", c_double_p), ("tsr_mode", C.c_int32), ("tsr_n", C.c_int32),
                ("tsr_sx", c_double_p), ("tsr_sy", c_double_p), ("tsr_sz", c_double_p), ("tsr_wdt", c_double_p),
                ("tsr_den", C.c_double)]


ET_OUT = ["t_prcp", "t_temp", "t_lai", "t_mf", "t_rn", "t_wind", "t_rh", "qEleprep", "qPotEvap", "qPotTran",
          "qEleETP", "qEleNetPrep", "qEleE_IC", "yEleIS", "yEleSnow", "fu_surf", "fu_sub", "rn_factor"]


class ShudEtOut(C.Structure):
    _fields_ = [(n, c_double_p) for n in ET_OUT]


# ---- include/shud_ode.h (device-resident integrator) ----
class ShudOdeOptions(C.Structure):
    _fields_ = [("reltol", C.c_double), ("abstol", C.c_double), ("init_step", C.c_double), ("max_step", C.c_double),
                ("min_step", C.c_double), ("max_num_steps", C.c_int64), ("maxl", C.c_int32), ("max_order", C.c_int32)]


ODE_STATS_I = ["nst", "nfe", "nfe_ls", "nni", "ncfn", "nnf", "netf", "nsetups", "nli", "ncfl", "njtimes"]


class ShudOdeStats(C.Structure):
    _fields_ = ([(n, C.c_int64) for n in ODE_STATS_I] + [("qlast", C.c_int32), ("qcur", C.c_int32)] +
                [(n, C.c_double) for n in ["hlast", "hcur", "tcur", "hnext"]] + [("n_sync", C.c_int64)])


ODE_SUCCESS, ODE_TSTOP_RETURN, ODE_RHSFUNC_FAIL = 0, 1, -8
ODE_NORMAL, ODE_ONE_STEP = 1, 2
OdeRhsFn = C.CFUNCTYPE(C.c_int, C.c_double, C.c_void_p, C.c_void_p, C.c_void_p)

# functions declared in include/shud_rhs.h (name -> (restype, argtypes))
_H = C.c_void_p
FUNCTIONS = {
    "shud_rhs_abi_version": (C.c_int, []),
    "shud_rhs_create": (C.c_int, [C.POINTER(ShudMeshSoA), C.POINTER(ShudParamsSoA), C.POINTER(ShudRhsOptions),
                                  C.POINTER(_H)]),
    "shud_rhs_set_step_inputs": (C.c_int, [_H, C.POINTER(ShudStepInputs)]),
    "shud_rhs_eval": (C.c_int, [_H, C.c_double, C.c_void_p, C.c_void_p, C.c_int]),
    "shud_rhs_sync_diagnostics": (C.c_int, [_H, C.POINTER(ShudFluxOut)]),
    "shud_rhs_get_error": (C.c_int, [_H, C.POINTER(ShudErr)]),
    "shud_rhs_clear_error": (C.c_int, [_H]),
    "shud_rhs_num_calls": (C.c_longlong, [_H]),
    "shud_rhs_layout": (C.c_int, [_H, C.POINTER(C.c_int), C.POINTER(C.c_int)]),
    "shud_rhs_layout_streamed": (C.c_int, [_H, C.POINTER(C.c_int)]),
    "shud_rhs_layout_shared": (C.c_int, [_H, C.POINTER(C.c_int)]),
    "shud_rhs_destroy": (C.c_int, [_H]),
    "shud_rhs_last_error_string": (C.c_char_p, []),
    "shud_rhs_cvrhs": (C.c_int, [C.c_double, C.c_void_p, C.c_void_p, C.c_void_p]),
    "shud_rhs_device_alloc": (C.c_int, [_H, C.c_size_t, C.POINTER(C.c_void_p)]),
    "shud_rhs_device_free": (C.c_int, [_H, C.c_void_p]),
    "shud_rhs_memcpy": (C.c_int, [_H, C.c_void_p, C.c_void_p, C.c_size_t, C.c_int]),
    "shud_rhs_synchronize": (C.c_int, [_H]),
    "shud_rhs_stream": (C.c_void_p, [_H]),
    "shud_rhs_time_kernels": (C.c_int, [_H, C.c_double, C.c_void_p, C.c_void_p, C.c_int, c_double_p, c_double_p,
                                        C.POINTER(C.c_int), C.c_char_p, C.c_int]),
    "shud_rhs_timing": (C.c_int, [_H, C.c_int, C.c_int]),
    "shud_rhs_timing_read": (C.c_int, [_H, c_double_p, c_double_p, c_double_p, C.POINTER(C.c_int)]),
    "shud_rhs_nccl_unique_id": (C.c_int, [C.c_char_p]),
    "shud_rhs_create_partitioned": (C.c_int, [C.POINTER(ShudMeshSoA), C.POINTER(ShudParamsSoA),
                                              C.POINTER(ShudRhsOptions), C.POINTER(ShudPartition),
                                              C.POINTER(_H)]),
    "shud_rhs_halo_buffers": (C.c_int, [_H, C.POINTER(C.c_void_p), C.POINTER(C.c_void_p), C.POINTER(C.c_void_p),
                                        C.POINTER(C.c_void_p)]),
    "shud_rhs_eval_pack": (C.c_int, [_H, C.c_void_p]),
    "shud_rhs_eval_compute": (C.c_int, [_H, C.c_double, C.c_void_p, C.c_void_p]),
    "shud_rhs_debug_halo": (C.c_int, [_H, C.c_double, C.c_void_p, C.c_void_p, C.c_int, C.c_double]),
}
# include/shud_et.h
ET_FUNCTIONS = {
    "shud_et_attach": (C.c_int, [_H, C.POINTER(ShudEtMeshSoA), C.POINTER(ShudEtParams)]),
    "shud_et_set_state": (C.c_int, [_H, C.c_void_p, C.c_void_p]),
    "shud_et_step": (C.c_int, [_H, C.POINTER(ShudEtForcing)]),
    "shud_et_get": (C.c_int, [_H, C.POINTER(ShudEtOut)]),
}

# include/shud_ode.h
ODE_FUNCTIONS = {
    "shud_ode_create": (C.c_int, [_H, C.c_double, C.c_void_p, C.c_int, C.POINTER(ShudOdeOptions), C.POINTER(_H)]),
    "shud_ode_create_fn": (C.c_int, [C.c_int64, C.c_void_p, C.c_void_p, C.c_void_p, C.c_double, C.c_void_p, C.c_int,
                                     C.POINTER(ShudOdeOptions), C.POINTER(_H)]),
    "shud_ode_set_stop_time": (C.c_int, [_H, C.c_double]),
    "shud_ode_solve": (C.c_int, [_H, C.c_double, C.c_void_p, C.c_int, C.POINTER(C.c_double), C.c_int]),
    "shud_ode_get_dky": (C.c_int, [_H, C.c_double, C.c_int, C.c_void_p, C.c_int]),
    "shud_ode_get_stats": (C.c_int, [_H, C.POINTER(ShudOdeStats)]),
    "shud_ode_state_device": (C.c_void_p, [_H]),
    "shud_ode_destroy": (C.c_int, [_H]),
}

# ---- include/shud_out.h (output path on the device) ----
(SHUD_ARR_Y_ELE_SURF, SHUD_ARR_Y_ELE_UNSAT, SHUD_ARR_Y_ELE_GW, SHUD_ARR_Y_RIV_STG, SHUD_ARR_Y_LAKE_STG,
 SHUD_ARR_QELE_SURF_TOT, SHUD_ARR_QELE_SUB_TOT, SHUD_ARR_QELE_SURF, SHUD_ARR_QELE_SUB, SHUD_ARR_QE2R_SURF,
 SHUD_ARR_QE2R_SUB, SHUD_ARR_Q_INFIL, SHUD_ARR_Q_EXFIL, SHUD_ARR_Q_RECHARGE, SHUD_ARR_Q_ETA, SHUD_ARR_Q_E_IC,
 SHUD_ARR_Q_TRANS, SHUD_ARR_Q_EVAPO, SHUD_ARR_QRIV_DOWN, SHUD_ARR_QRIV_UP, SHUD_ARR_QRIV_SURF, SHUD_ARR_QRIV_SUB,
 SHUD_ARR_Q_PRCP, SHUD_ARR_Q_NET_PRCP, SHUD_ARR_Q_ETP, SHUD_ARR_Y_ELE_IS, SHUD_ARR_Y_ELE_SNOW, SHUD_ARR_RN_H,
 SHUD_ARR_RN_T, SHUD_ARR_RN_FACTOR, SHUD_ARR_LAKE_TOPAREA, SHUD_ARR_Q_LAKE_EVAP, SHUD_ARR_Q_LAKE_PRCP,
 SHUD_ARR_Q_LAKE_RIVIN, SHUD_ARR_Q_LAKE_RIVOUT, SHUD_ARR_Q_LAKE_SURF, SHUD_ARR_Q_LAKE_SUB, SHUD_ARR_COUNT) = range(38)


class ShudPrintSpec(C.Structure):
    _fields_ = [("basename", C.c_char_p), ("d_src", C.c_void_p), ("n_all", C.c_int32), ("flag_io", C.c_void_p),
                ("interval", C.c_int32), ("iflux", C.c_int32), ("start_time", C.c_int64), ("binary", C.c_int32),
                ("ascii", C.c_int32), ("radiation_input_mode", C.c_int32), ("terrain_radiation", C.c_int32),
                ("solar_lonlat_mode", C.c_char_p), ("solar_lon_deg", C.c_double), ("solar_lat_deg", C.c_double)]


OUT_FUNCTIONS = {
    "shud_rhs_summary": (C.c_int, [_H, C.c_void_p]),
    "shud_rhs_refresh_diagnostics": (C.c_int, [_H]),
    "shud_rhs_prepare_outputs": (C.c_int, [_H]),
    "shud_rhs_device_array": (C.c_void_p, [_H, C.c_int, C.POINTER(C.c_int64)]),
    "shud_out_create": (C.c_int, [C.c_int, C.c_void_p, C.POINTER(_H)]),
    "shud_out_add": (C.c_int, [_H, C.POINTER(ShudPrintSpec)]),
    "shud_out_export": (C.c_int, [_H, C.c_double]),
    "shud_out_rows": (C.c_int64, [_H, C.c_int]),
    "shud_out_flush": (C.c_int, [_H]),
    "shud_out_destroy": (C.c_int, [_H]),
}


def bind(lib, strict=True):
    """set the signatures; strict=False (A/B builds of older sources) skips symbols the library lacks"""
    for name, (res, args) in (list(FUNCTIONS.items()) + list(ET_FUNCTIONS.items()) + list(ODE_FUNCTIONS.items())
                              + list(OUT_FUNCTIONS.items())):
        if not strict and not hasattr(lib, name):
            continue
        f = getattr(lib, name)
        f.restype = res
        f.argtypes = args
    return lib
