# BatchReactorHIP.jl -- the Julia host side a BatchReactor.jl maintainer would add: `ccall`
# bindings of libbrhip.so (include/brhip.h). Julia is not installed in the build image, so this file
# is not executed here; every struct below mirrors its C counterpart field for field (same order,
# same C types), and the Python host (batchreactor.jl_amd/_lib.py) binds the same layout and is
# tested. Replaces, per reactor, `solve(ODEProblem(residual!, u0, (0, tf), params), CVODE_BDF();
# reltol=1e-6, abstol=1e-10)` of src/BatchReactor.jl:138-141,:204-210.
module BatchReactorHIP

using Printf

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
    dq_jacobian::Cint           # 1: CVODE's DQ Jacobian (cvLsDenseDQJac, the reference's setting), every engine
end
# dq_jacobian=true selects CVODE's difference-quotient Jacobian, the reference's CVODE_BDF() setting
# (src/BatchReactor.jl:140,:204); the default is the analytic Jacobian
BrOpts(; rtol=1e-6, atol=1e-10, max_steps=100_000, device=0, hmax=0.0, unstable_factor=0.0, ignition_species=0,
       dq_jacobian::Bool=false) =
    BrOpts(rtol, atol, Cint(max_steps), Cint(device), Float64(hmax), Cint(0), Float64(unstable_factor),
           Cint(ignition_species), Cint(0), C_NULL, C_NULL, Cint(dq_jacobian))

# br_stats rows of the [NSTAT x N] matrix returned below
const STAT_FIELDS = (:nsteps, :nfe, :nje, :nsetups, :nni, :ncfn, :netf, :status, :cyc_total, :cyc_rhs, :cyc_jac,
                     :cyc_lu, :cyc_sol, :t_end, :cyc_ctl, :cyc_clk, :t_ign, :ign_rate, :ign_dt, :nfe_dq)

last_error() = unsafe_string(ccall((:br_last_error, lib), Cstring, ()))
check(rc) = rc == 0 || error("libbrhip error $rc: " * last_error())

"""Create the device-resident mechanism (br_mech_create). `desc` (and the arrays it points to) must
stay alive for the call; the handle copies the tables to the GPU."""
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

# ---------------------------------------------------------------------------------------------
# host mechanism compiler and batch.xml reader of libbrhip.so (C++; br_mech_parse, br_read_batch_xml):
# the Julia host needs no Python and no chemistry package to build the tables
# ---------------------------------------------------------------------------------------------
const R_GAS = 8.31446261815324        # RxnHelperUtils.R (src/BatchReactor.jl:338)

"""A mechanism compiled on the host (tables, species names, molecular weights, initial coverages)
and its device-resident copy on one GPU (br_mech)."""
mutable struct DeviceMech
    host::Ptr{Cvoid}                   # br_host_mech (owns the br_mech_desc arrays)
    m::Ptr{Cvoid}                      # br_mech on `device`
    device::Int
    ng::Int; ns::Int; nrg::Int; nrs::Int
    species::Vector{String}            # gas species (mechanism order), then surface species
    molwt::Vector{Float64}             # [ng] kg/mol
    theta0::Vector{Float64}            # [ns]
end
ncomp(dm::DeviceMech) = dm.ng + dm.ns
gas_species(dm::DeviceMech) = dm.species[1:dm.ng]
surf_species(dm::DeviceMech) = dm.species[dm.ng+1:end]

function _free!(dm::DeviceMech)
    dm.m != C_NULL && ccall((:br_mech_destroy, lib), Cint, (Ptr{Cvoid},), dm.m)
    dm.host != C_NULL && ccall((:br_host_mech_free, lib), Cint, (Ptr{Cvoid},), dm.host)
    dm.m = C_NULL
    dm.host = C_NULL
    return nothing
end

"""compile_gaschemistry + IdealGas.create_thermo + SurfaceReactions.compile_mech
(src/BatchReactor.jl:242-287) through br_mech_parse, then br_mech_create on `device`.
`gas_mech == ""`: surface-only run, gas species from `gasphase` (space-separated, the <gasphase> tag)."""
function compile_mechanism(gas_mech::AbstractString, therm::AbstractString, surf_mech::AbstractString="";
                           gasphase::AbstractString="", conv::Integer=CONV_REFERENCE, device::Integer=0)
    h, d, names, molwt, theta0 = _parse_host(gas_mech, therm, surf_mech; gasphase=gasphase, conv=conv)
    m = C_NULL
    try
        m = mech_create(d, device)
        dd = d[]
        dm = DeviceMech(h, m, Int(device), Int(dd.ng), Int(dd.ns), Int(dd.nrg), Int(dd.nrs), names, molwt, theta0)
        finalizer(_free!, dm)
        return dm
    catch
        m != C_NULL && ccall((:br_mech_destroy, lib), Cint, (Ptr{Cvoid},), m)
        ccall((:br_host_mech_free, lib), Cint, (Ptr{Cvoid},), h)
        rethrow()
    end
end

"""The host half of compile_mechanism (br_mech_parse; no GPU): the br_host_mech handle (the caller
frees it with br_host_mech_free), its br_mech_desc, species names, molecular weights and theta0."""
function _parse_host(gas_mech::AbstractString, therm::AbstractString, surf_mech::AbstractString="";
                     gasphase::AbstractString="", conv::Integer=CONV_REFERENCE)
    h = Ref{Ptr{Cvoid}}(C_NULL)
    check(ccall((:br_mech_parse, lib), Cint, (Cstring, Cstring, Cstring, Cstring, Cint, Ref{Ptr{Cvoid}}),
                gas_mech, therm, surf_mech, gasphase, conv, h))
    # every step after br_mech_parse may throw (check): free the handle, then rethrow
    try
        d = Ref{BrMechDesc}()
        check(ccall((:br_host_mech_desc, lib), Cint, (Ptr{Cvoid}, Ref{BrMechDesc}), h[], d))
        ng, ns = Int(d[].ng), Int(d[].ns)
        buf = zeros(UInt8, 64)
        names = String[]
        for i in 0:(ng + ns - 1)
            check(ccall((:br_host_mech_species, lib), Cint, (Ptr{Cvoid}, Cint, Ptr{UInt8}, Csize_t), h[], i, buf, 64))
            push!(names, unsafe_string(pointer(buf)))
        end
        molwt = copy(unsafe_wrap(Array, d[].molwt, ng))
        theta0 = zeros(ns)
        check(ccall((:br_host_mech_theta0, lib), Cint, (Ptr{Cvoid}, Ptr{Float64}), h[], theta0))
        return h[], d, names, molwt, theta0
    catch
        ccall((:br_host_mech_free, lib), Cint, (Ptr{Cvoid},), h[])
        rethrow()
    end
end

# br_batch_input (br_read_batch_xml)
const BATCH_MAXCOMP = 64
struct BrBatchInput
    gas_mech::NTuple{256,UInt8}
    surface_mech::NTuple{256,UInt8}
    gasphase::NTuple{1024,UInt8}
    T::Float64; p::Float64; Asv::Float64; time::Float64
    has_T::Cint; has_p::Cint; has_Asv::Cint; has_time::Cint
    ncomp::Cint; comp_is_mass::Cint
    comp_names::NTuple{BATCH_MAXCOMP,NTuple{32,UInt8}}
    comp_values::NTuple{BATCH_MAXCOMP,Float64}
end
function _cstr(t)
    v = collect(t)
    k = findfirst(==(0x00), v)
    return String(v[1:(k === nothing ? length(v) : k - 1)])
end

"""input_data's view of batch.xml (src/BatchReactor.jl:238-306): a missing <Asv> reads as 1."""
function read_batch_xml(path::AbstractString)
    b = Ref{BrBatchInput}()
    check(ccall((:br_read_batch_xml, lib), Cint, (Cstring, Ref{BrBatchInput}), path, b))
    x = b[]
    comp = Dict{String,Float64}(_cstr(x.comp_names[i]) => x.comp_values[i] for i in 1:Int(x.ncomp))
    return (gas_mech=_cstr(x.gas_mech), surface_mech=_cstr(x.surface_mech), gasphase=_cstr(x.gasphase),
            T=x.T, p=x.p, Asv=x.Asv, time=x.time, comp=comp, comp_is_mass=x.comp_is_mass != 0)
end

"""get_solution_vector (src/BatchReactor.jl:224-232): u0 = [rho*Y_k ; theta0] from mole (or mass)
fractions by species name; rho0 = p Mbar / (R T)."""
function initial_state(dm::DeviceMech, T::Real, p::Real, comp::AbstractDict; is_mass::Bool=false,
                       theta::Union{Nothing,AbstractVector}=nothing)
    ng = dm.ng
    v = zeros(ng)
    for (k, val) in comp
        i = findfirst(==(uppercase(String(k))), gas_species(dm))
        i === nothing && continue
        v[i] = val
    end
    x = is_mass ? (t = v ./ dm.molwt; t ./ sum(t)) : v
    Mb = sum(x .* dm.molwt)
    rho = p * Mb / (R_GAS * T)
    u = zeros(ncomp(dm))
    u[1:ng] .= (x .* dm.molwt ./ Mb) .* rho
    u[ng+1:end] .= theta === nothing ? dm.theta0 : theta
    return u
end

"""Final conversion (src/BatchReactor.jl:142-144): Y = u / sum(u) over the gas species -> x."""
function state_to_molefrac(dm::DeviceMech, u::AbstractVector)
    y = u[1:dm.ng] ./ sum(u[1:dm.ng])
    t = y ./ dm.molwt
    return t ./ sum(t)
end

ignition_species(dm::DeviceMech) = something(findfirst(==("OH"), gas_species(dm)), 0)

# ---- save_data (src/BatchReactor.jl:383-402): RxnHelperUtils' .dat (%10s / %.4e, TAB) and .csv
#      (string(::Float64)) rows; x, p and coverages of the step's last RHS evaluation, rho from u
function _write_profiles(folder, dm::DeviceMech, surf::Bool, T, trace, nst)
    n, ng = ncomp(dm), dm.ng
    g_dat = open(joinpath(folder, "gas_profile.dat"), "w")
    s_dat = open(joinpath(folder, "surface_covg.dat"), "w")
    g_csv = open(joinpath(folder, "gas_profile.csv"), "w")
    s_csv = open(joinpath(folder, "surface_covg.csv"), "w")
    try
        hdr = vcat(["t", "T", "p", "rho"], gas_species(dm))
        write(g_dat, join([@sprintf("%10s\t", h) for h in hdr]), "\n")
        write(g_csv, join(hdr, ","), "\n")
        if surf
            sh = vcat(["t", "T"], surf_species(dm))
            write(s_dat, join([@sprintf("%10s\t", h) for h in sh]), "\n")
            write(s_csv, join(sh, ","), "\n")
        end
        for k in 0:nst
            row = trace[:, k + 1, 1]
            u, y = row[5:4+n], row[5+n:4+2n]
            vals = vcat([row[1], T, row[4], sum(u[1:ng])], state_to_molefrac(dm, y))
            write(g_dat, join([@sprintf("%.4e\t", v) for v in vals]), "\n")
            write(g_csv, join(string.(vals), ","), "\n")
            if surf
                sv = vcat([row[1], T], y[ng+1:n])
                write(s_dat, join([@sprintf("%.4e\t", v) for v in sv]), "\n")
                write(s_csv, join(string.(sv), ","), "\n")
            end
        end
    finally
        close(g_dat); close(s_dat); close(g_csv); close(s_csv)
    end
end

"""batch_reactor(input_file, lib_dir; sens, surfchem, gaschem) (src/BatchReactor.jl:67-70,:152-217)
on the HIP engine: reads batch.xml, compiles the mechanism library files natively, integrates the
reactor (CVODE_BDF restatement, rtol 1e-6, atol 1e-10), writes gas_profile.{dat,csv} and
surface_covg.{dat,csv} next to the input and returns Symbol(retcode). sens=true returns
(params, prob, t_span) with prob.f = residual! evaluated on the GPU (br_rhs). dq_jacobian=true
runs CVODE's difference-quotient Jacobian, the reference's own CVODE_BDF() setting (:204-210);
the default is the analytic Jacobian (same step-control algorithm)."""
function batch_reactor(input_file::AbstractString, lib_dir::AbstractString; sens::Bool=false,
                       surfchem::Bool=false, gaschem::Bool=false, device::Integer=0,
                       conv::Integer=CONV_REFERENCE, max_steps::Integer=100_000, dq_jacobian::Bool=false)
    inp = read_batch_xml(input_file)
    gm = gaschem ? joinpath(lib_dir, inp.gas_mech) : ""
    sm = surfchem ? joinpath(lib_dir, inp.surface_mech) : ""
    dm = compile_mechanism(gm, joinpath(lib_dir, "therm.dat"), sm; gasphase=gaschem ? "" : inp.gasphase,
                           conv=conv, device=device)
    u0 = initial_state(dm, inp.T, inp.p, inp.comp; is_mass=inp.comp_is_mass)
    n = ncomp(dm)
    if sens
        residual! = (du, u, p, t) -> (du .= rhs(dm, inp.T, inp.Asv, u); nothing)
        params = (thermo=dm, cp=(Asv=inp.Asv, T=inp.T), chem=(surfchem=surfchem, gaschem=gaschem))
        t_span = (0.0, inp.time)
        return params, (f=residual!, u0=u0, tspan=t_span, p=params), t_span
    end
    opts = BrOpts(max_steps=max_steps, ignition_species=ignition_species(dm), dq_jacobian=dq_jacobian)
    cap = min(4096, max_steps)
    stats, trace = integrate_traced!(dm.m, [inp.T], [inp.Asv], reshape(copy(u0), n, 1), [inp.time]; cap=cap, opts=opts)
    nst = Int(stats[1, 1])
    if nst > cap   # deterministic: the repeat takes the same steps
        stats, trace = integrate_traced!(dm.m, [inp.T], [inp.Asv], reshape(copy(u0), n, 1), [inp.time]; cap=nst,
                                         opts=opts)
        nst = Int(stats[1, 1])
    end
    _write_profiles(dirname(abspath(input_file)), dm, surfchem, inp.T, trace, nst)
    _free!(dm)
    return retcode_symbol(stats[8, 1])
end

"""Symbol(sol.retcode) of the reference's CVODE_BDF solve (src/BatchReactor.jl:216) for an engine status
(include/brhip.h): as Sundials.jl's interpret_sundials_retcode, -1 (CV_TOO_MUCH_WORK) -> :MaxIters,
-2 / -3 (CV_TOO_MUCH_ACC, CV_ERR_FAILURE) -> :Unstable, -4 (CV_CONV_FAILURE) -> :ConvergenceFailure,
other failures -> :Failure; a NaN state (SciML's unstable_check, status -7) -> :Unstable. The same
table as the Python host's reactor.RETCODES."""
function retcode_symbol(status::Real)
    s = Int(status)
    s == 0 && return :Success
    s == -1 && return :MaxIters
    (s == -2 || s == -3 || s == -7) && return :Unstable
    s == -4 && return :ConvergenceFailure
    return :Failure
end

"""residual!(du, u, p, t) (src/BatchReactor.jl:312-376) of one reactor on the GPU (br_rhs)."""
function rhs(dm::DeviceMech, T::Real, Asv::Real, u::AbstractVector)
    du = zeros(length(u))
    check(ccall((:br_rhs, lib), Cint, (Ptr{Cvoid}, Cint, Ptr{Float64}, Ptr{Float64}, Ptr{Float64}, Ptr{Float64}),
                dm.m, 1, [Float64(T)], [Float64(Asv)], collect(Float64, u), du))
    return du
end

"""batch_reactor(inlet_comp, T, p, time; Asv, chem, thermo_obj, md) (src/BatchReactor.jl:86-147):
returns (t = [0, time], Dict(species => x_end)); the mechanism is a DeviceMech from compile_mechanism.
`chem` is the reference's Chemistry(surfchem, gaschem, userchem, udf) (ReactionCommons) or this
module's `Chemistry`: any object with `surfchem` / `gaschem` fields; the flags must describe `md`
(gas reactions present iff gaschem, surface species present iff surfchem; the reference takes one
chemistry per call, :102-127). `thermo_obj` (IdealGas.SpeciesThermoObj in the reference, :131) is
accepted for call compatibility: `md` carries the NASA-7 tables and molecular weights of the same
species, matched by name. dq_jacobian as in the file-driven method."""
function batch_reactor(inlet_comp::AbstractDict, T::Real, p::Real, time::Real; Asv::Real=1.0, chem=nothing,
                       thermo_obj=nothing, md::DeviceMech, dq_jacobian::Bool=false)
    if chem !== nothing
        sc, gc = Bool(getproperty(chem, :surfchem)), Bool(getproperty(chem, :gaschem))
        (sc || gc) || error("chem: neither surfchem nor gaschem is set")
        gc == (md.nrg > 0) || error("chem.gaschem = $gc but the mechanism has $(md.nrg) gas reactions")
        sc == (md.ns > 0) || error("chem.surfchem = $sc but the mechanism has $(md.ns) surface species")
    end
    u = reshape(initial_state(md, T, p, inlet_comp), ncomp(md), 1)
    stats = integrate!(md.m, [Float64(T)], [Float64(Asv)], u, [Float64(time)]; opts=BrOpts(dq_jacobian=dq_jacobian))
    # as the reference (which does not check sol.retcode here): a failed solve still returns, t ending
    # at the time reached and x from the last accepted state
    tend = stats[8, 1] == 0 ? Float64(time) : stats[14, 1]
    xf = Dict(zip(gas_species(md), state_to_molefrac(md, u[:, 1])))
    if md.nrg == 0 && md.ns > 0   # surfchem: species = collect(keys(inlet_comp)) (:103, :145)
        return [0.0, tend], Dict(String(k) => xf[uppercase(String(k))] for k in keys(inlet_comp))
    end
    return [0.0, tend], xf
end

"""batch_reactor_ensemble: N independent reactors, each with its own T, p, inlet composition and
end time, in one call (one br_integrate over the ensemble). Returns (x_end [ng x N], theta_end
[ns x N], stats [NSTAT x N], including t_ign from the OH marker)."""
function batch_reactor_ensemble(md::DeviceMech, T::AbstractVector, p::AbstractVector, comps::AbstractVector,
                                tf; Asv=1.0, rtol::Real=1e-6, atol::Real=1e-10)
    N = length(T)
    U = zeros(ncomp(md), N)
    for i in 1:N
        U[:, i] = initial_state(md, T[i], p[i], comps[i])
    end
    fillv(v) = v isa AbstractVector ? collect(Float64, v) : fill(Float64(v), N)
    opts = BrOpts(rtol=rtol, atol=atol, ignition_species=ignition_species(md))
    stats = integrate!(md.m, collect(Float64, T), fillv(Asv), U, fillv(tf); opts=opts)
    X = reduce(hcat, [state_to_molefrac(md, U[:, i]) for i in 1:N])
    return X, U[md.ng+1:end, :], stats
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

# ---------------------------------------------------------------------------------------------
# user-defined chemistry (src/BatchReactor.jl:42-54, :197-200, :358-360, :371-372)
# ---------------------------------------------------------------------------------------------
"""ReactionCommons.Chemistry(surfchem, gaschem, userchem, udf) (src/BatchReactor.jl:52,:68)."""
struct Chemistry
    surfchem::Bool
    gaschem::Bool
    userchem::Bool
    udf::Function
end

"""ReactionCommons.UserDefinedState(T, p, mole_frac, molwt, species, source) as the reference builds
it (:197-200): the udf fills `source` [mol/m3/s]; du = source .* molwt (:371-372)."""
mutable struct UserDefinedState
    T::Float64
    p::Float64
    mole_frac::Vector{Float64}
    molwt::Vector{Float64}
    species::Vector{String}
    source::Vector{Float64}
end

"""The state handed to the user's function: ReactionCommons.UserDefinedState when the caller has that
package loaded (the reference's own type, built with the reference's arguments, src/BatchReactor.jl:
197-200, so a udf annotated with it dispatches), else this module's struct with the same fields."""
function _udf_state(T, p, x, molwt, names, source)
    if isdefined(Main, :ReactionCommons) && isdefined(getfield(Main, :ReactionCommons), :UserDefinedState)
        return getfield(getfield(Main, :ReactionCommons), :UserDefinedState)(T, p, x, molwt, names, source)
    end
    return UserDefinedState(T, p, x, molwt, names, source)
end

mutable struct _HostCtx
    n::Int
    f!::Any          # f!(du, u, t)
    rowcb::Any       # rowcb(t, u)
    err::Any
end

# br_integrate_host callbacks: the user's residual! and save_data's row per accepted step
function _host_rhs(user::Ptr{Cvoid}, t::Cdouble, u::Ptr{Cdouble}, du::Ptr{Cdouble})::Cint
    ctx = unsafe_pointer_to_objref(user)::_HostCtx
    try
        ctx.f!(unsafe_wrap(Array, du, ctx.n), copy(unsafe_wrap(Array, u, ctx.n)), t)
        return Cint(0)
    catch e
        ctx.err = e
        return Cint(1)                                                  # -> BR_ERR_RHS
    end
end
function _host_step(user::Ptr{Cvoid}, t::Cdouble, u::Ptr{Cdouble})::Cvoid
    ctx = unsafe_pointer_to_objref(user)::_HostCtx
    ctx.err === nothing && ctx.rowcb(t, copy(unsafe_wrap(Array, u, ctx.n)))
    return nothing
end

"""CVODE_BDF() on the host with a Julia right-hand side f!(du, u, t) (br_integrate_host: the engine's
CVODE 5.x restatement with CVODE's DQ Jacobian, the reference's setting, src/BatchReactor.jl:204-210;
the same solver the Python host's udf path calls). rowcb(t, u) after every accepted step and at
t = 0 / tf (save_data's rows, :208). Returns (status, u_end, stats); an exception in f! is rethrown."""
function integrate_host(f!, u0::Vector{Float64}, tf::Float64; rtol=1e-6, atol=1e-10, max_steps=100_000,
                        rowcb=(t, u) -> nothing)
    ctx = _HostCtx(length(u0), f!, rowcb, nothing)
    u = copy(u0)
    stats = zeros(NSTAT)
    frhs = @cfunction(_host_rhs, Cint, (Ptr{Cvoid}, Cdouble, Ptr{Cdouble}, Ptr{Cdouble}))
    fstep = @cfunction(_host_step, Cvoid, (Ptr{Cvoid}, Cdouble, Ptr{Cdouble}))
    status = GC.@preserve ctx begin
        p = pointer_from_objref(ctx)
        ccall((:br_integrate_host, lib), Cint,
              (Cint, Ptr{Cvoid}, Ptr{Cvoid}, Ptr{Float64}, Cdouble, Cdouble, Cdouble, Cint, Ptr{Cvoid}, Ptr{Cvoid},
               Ptr{Float64}),
              length(u0), frhs, p, u, tf, rtol, atol, max_steps, fstep, p, stats)
    end
    ctx.err === nothing || throw(ctx.err)
    return status, u, stats
end

"""batch_reactor(input_file, lib_dir, user_defined::Function; sens=false) (src/BatchReactor.jl:51-54):
user-defined chemistry. The gas species are batch.xml's <gasphase> (no mechanism files, :256-260;
molecular weights from lib_dir/therm.dat through br_mech_parse, no GPU). The udf is called with a
UserDefinedState whose T, p and mole fractions stay at the inlet values, as in the reference; its
`source` drives du = source .* molwt. Host code by nature (a Julia callback cannot run in a HIP
kernel): integrated by CVODE_BDF on the host (integrate_host -> br_integrate_host, as the reference's
solve at :204-210), one output row per accepted step in the save_data format (t, T, p, rho = sum(u),
the state's mole fractions; :383-402). Returns Symbol(retcode). sens=true returns (params, prob, t_span)
with prob.f = residual! (:205-207)."""
function batch_reactor(input_file::AbstractString, lib_dir::AbstractString, user_defined::Function;
                       sens::Bool=false, max_steps::Integer=100_000)
    inp = read_batch_xml(input_file)
    h, _, names, molwt, _ = _parse_host("", joinpath(lib_dir, "therm.dat"), ""; gasphase=inp.gasphase)
    ccall((:br_host_mech_free, lib), Cint, (Ptr{Cvoid},), h)
    ng = length(names)
    v = zeros(ng)
    for (k, val) in inp.comp
        i = findfirst(==(uppercase(String(k))), names)
        i === nothing || (v[i] = val)
    end
    x = inp.comp_is_mass ? (t = v ./ molwt; t ./ sum(t)) : v
    Mb = sum(x .* molwt)
    rho = inp.p * Mb / (R_GAS * inp.T)
    u0 = (x .* molwt ./ Mb) .* rho                                          # get_solution_vector (:224-232)
    state = _udf_state(inp.T, inp.p, copy(x), molwt, names, zeros(ng))
    chem = Chemistry(false, false, true, user_defined)
    residual! = (du, u, p, t) -> (user_defined(state); du[1:ng] .= state.source[1:ng] .* molwt; nothing)
    if sens
        params = (s_state=nothing, g_state=nothing, u_state=state, thermo=(molwt=molwt, species=names),
                  smd=nothing, gmd=nothing, cp=(Asv=inp.Asv, T=inp.T), chem=chem)
        t_span = (0.0, inp.time)
        return params, (f=residual!, u0=u0, tspan=t_span, p=params), t_span
    end
    folder = dirname(abspath(input_file))
    g_dat = open(joinpath(folder, "gas_profile.dat"), "w")
    s_dat = open(joinpath(folder, "surface_covg.dat"), "w")
    g_csv = open(joinpath(folder, "gas_profile.csv"), "w")
    s_csv = open(joinpath(folder, "surface_covg.csv"), "w")
    status = 0
    try
        hdr = vcat(["t", "T", "p", "rho"], names)
        write(g_dat, join([@sprintf("%10s\t", hh) for hh in hdr]), "\n")
        write(g_csv, join(hdr, ","), "\n")
        row = (t, u) -> begin
            vals = vcat([t, state.T, state.p, sum(u)], state.mole_frac)
            write(g_dat, join([@sprintf("%.4e\t", vv) for vv in vals]), "\n")
            write(g_csv, join(string.(vals), ","), "\n")
        end
        f! = (du, u, t) -> residual!(du, u, nothing, t)
        status, _, _ = integrate_host(f!, u0, Float64(inp.time); max_steps=max_steps, rowcb=row)
    finally
        close(g_dat); close(s_dat); close(g_csv); close(s_csv)
    end
    return retcode_symbol(status)
end

export batch_reactor, batch_reactor_ensemble, compile_mechanism, read_batch_xml, DeviceMech, Chemistry,
       UserDefinedState, BrOpts, retcode_symbol, integrate_host

end # module
