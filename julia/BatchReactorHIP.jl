# BatchReactorHIP.jl -- the Julia host side a BatchReactor.jl maintainer would add: `ccall`
# bindings of libbrhip.so (include/brhip.h). Julia is not installed in the build image, so this file
# is not executed here; every struct below mirrors its C counterpart field for field (same order,
# same C types), and the Python host (batchreactor.jl_amd/_lib.py) binds the same layout and is
# tested. Replaces, per reactor, `solve(ODEProblem(residual!, u0, (0, tf), params), CVODE_BDF();
# reltol=1e-6, abstol=1e-10)` of src/BatchReactor.jl:138-141,:204-210.
module BatchReactorHIP

const lib = joinpath(@__DIR__, "..", "batchreactor.jl_amd", "libbrhip.so")

# convention bits (br_mech_desc.conv); REFERENCE = what GasphaseReactions does (DESIGN.md section 1)
const CONV_KC_UNIT_SLIP = Cint(1)
const CONV_FALLOFF_XM   = Cint(2)
const CONV_DOC_COVG     = Cint(4)
const CONV_TROE_C4      = Cint(16)
const CONV_REFERENCE    = CONV_KC_UNIT_SLIP | CONV_FALLOFF_XM | CONV_TROE_C4
const NSTAT = 20                                   # BR_NSTAT

# br_mech_desc: flat SoA tables of the compiled mechanism (SI units, 0-based species indices)
struct BrMechDesc
    ng::Cint; ns::Cint; nrg::Cint; nrs::Cint
    conv::Cint
    p_std::Float64
    molwt::Ptr{Float64}        # [ng] kg/mol
    nasa::Ptr{Float64}         # [ng][15] Tmid, a_hi[7], a_lo[7]
    g_nf::Ptr{Cint}; g_nr::Ptr{Cint}
    g_f::Ptr{Cint}; g_r::Ptr{Cint}               # [nrg][4], -1 pad
    g_rev::Ptr{Cint}; g_tb::Ptr{Cint}            # [nrg]; tb 0 / 1 (+M) / 2 (+M) falloff
    g_arr::Ptr{Float64}                          # [nrg][3] A (SI), beta, Ea/R
    g_low::Ptr{Float64}                          # [nrg][3]
    g_troe_n::Ptr{Cint}; g_troe::Ptr{Float64}    # [nrg], [nrg][4]
    g_eff::Ptr{Float64}                          # [nrg][ng]
    site_density::Float64                        # mol/cm2
    sigma::Ptr{Float64}                          # [ns]
    s_nf::Ptr{Cint}; s_np::Ptr{Cint}
    s_f::Ptr{Cint}; s_p::Ptr{Cint}               # [nrs][6], combined index, -1 pad
    s_stick::Ptr{Cint}
    s_arr::Ptr{Float64}                          # [nrs][3] A (SI) or s0, beta, Ea [J/mol]
    s_ncov::Ptr{Cint}; s_cov_sp::Ptr{Cint}       # [nrs], [nrs][4]
    s_cov_eps::Ptr{Float64}                      # [nrs][4] J/mol
end

# br_opts
struct BrOpts
    rtol::Float64; atol::Float64
    max_steps::Cint; device::Cint
    hmax::Float64
    trace_cap::Cint
    unstable_factor::Float64
    ignition_species::Cint      # 1-based gas species index (OH) for br_stats.t_ign; 0 = off
    nout::Cint
    tout::Ptr{Float64}          # [nout] ascending output times
    yout::Ptr{Float64}          # [N][nout][n]
    dq_jacobian::Cint           # 1: CVODE's DQ Jacobian in the per-lane engine
end
BrOpts(; rtol=1e-6, atol=1e-10, max_steps=100_000, device=0, ignition_species=0) =
    BrOpts(rtol, atol, Cint(max_steps), Cint(device), 0.0, Cint(0), 0.0, Cint(ignition_species), Cint(0),
           C_NULL, C_NULL, Cint(0))

# br_stats rows of the [NSTAT x N] matrix returned below
const STAT_FIELDS = (:nsteps, :nfe, :nje, :nsetups, :nni, :ncfn, :netf, :status, :cyc_total, :cyc_rhs, :cyc_jac,
                     :cyc_lu, :cyc_sol, :t_end, :cyc_ctl, :cyc_clk, :t_ign, :ign_rate, :ign_dt, :reserved)

last_error() = unsafe_string(ccall((:br_last_error, lib), Cstring, ()))
check(rc) = rc == 0 || error("libbrhip error $rc: " * last_error())

"""Create the device-resident mechanism (br_mech_create). `desc` must stay alive for the call."""
function mech_create(desc::Ref{BrMechDesc}, device::Integer=0)
    h = Ref{Ptr{Cvoid}}(C_NULL)
    check(ccall((:br_mech_create, lib), Cint, (Ref{BrMechDesc}, Cint, Ref{Ptr{Cvoid}}), desc, device, h))
    return h[]
end
mech_destroy(m::Ptr{Cvoid}) = check(ccall((:br_mech_destroy, lib), Cint, (Ptr{Cvoid},), m))

"""N reactors 0 -> tf (br_integrate). `u` is n x N column-major in Julia, i.e. the reactor-major
[N][n] rows of the C layout; it is overwritten with the end states. Returns the NSTAT x N stats."""
function integrate!(m::Ptr{Cvoid}, T::Vector{Float64}, Asv::Vector{Float64}, u::Matrix{Float64},
                    tf::Vector{Float64}; opts::BrOpts=BrOpts())
    N = length(T)
    stats = zeros(NSTAT, N)
    check(ccall((:br_integrate, lib), Cint,
                (Ptr{Cvoid}, Cint, Ptr{Float64}, Ptr{Float64}, Ptr{Float64}, Ptr{Float64}, Ref{BrOpts}, Ptr{Float64}),
                m, N, T, Asv, u, tf, Ref(opts), stats))
    return stats
end

"""As integrate!, with the per-accepted-step rows save_data writes (src/BatchReactor.jl:383-402):
trace[2n+4, cap+1, N] = (t, h, q, p_last, u[1:n], y_last[1:n]) per row."""
function integrate_traced!(m::Ptr{Cvoid}, T, Asv, u::Matrix{Float64}, tf; cap::Integer=100_000, opts::BrOpts=BrOpts())
    n, N = size(u)
    stats = zeros(NSTAT, N)
    trace = zeros(2n + 4, cap + 1, N)
    o = BrOpts(opts.rtol, opts.atol, opts.max_steps, opts.device, opts.hmax, Cint(cap), opts.unstable_factor,
               opts.ignition_species, Cint(0), C_NULL, C_NULL, opts.dq_jacobian)
    check(ccall((:br_integrate_traced, lib), Cint,
                (Ptr{Cvoid}, Cint, Ptr{Float64}, Ptr{Float64}, Ptr{Float64}, Ptr{Float64}, Ref{BrOpts}, Ptr{Float64},
                 Ptr{Float64}), m, N, T, Asv, u, tf, Ref(o), stats, trace))
    return stats, trace
end

"""The ensemble over several GPUs (br_integrate_multi): `mechs[d]` created on device d."""
function integrate_multi!(mechs::Vector{Ptr{Cvoid}}, T, Asv, u::Matrix{Float64}, tf; opts::BrOpts=BrOpts())
    N = length(T)
    stats = zeros(NSTAT, N)
    check(ccall((:br_integrate_multi, lib), Cint,
                (Ptr{Ptr{Cvoid}}, Cint, Cint, Ptr{Float64}, Ptr{Float64}, Ptr{Float64}, Ptr{Float64}, Ref{BrOpts},
                 Ptr{Float64}), mechs, length(mechs), N, T, Asv, u, tf, Ref(opts), stats))
    return stats
end

end # module
