# PamgHIP.jl — Julia binding of libpamg (include/pamg.h), the host side BASELINE.json's
# north star asks for: a PartitionedArrays-based AMG code keeps its operator surface (mul!,
# consistent!, dot, norm, axpy!, ldiv! with a V-cycle preconditioner) and the work runs in the
# gfx950 kernels of libpamg.so over `ccall`.
#
# NOT runnable in this image (no Julia, no PartitionedArrays.jl, no network). What is tested
# here: every `ccall` below is parsed by tests/test_julia_binding.py and checked against the C
# prototypes of include/pamg.h (symbol, argument count, argument and return types), the same
# contract tests/test_abi.py checks for the Python binding. The PartitionedArrays adapter is the
# package extension ext/PamgHIPPartitionedArraysExt.jl.
#
# Conventions mirrored from the C-ABI: every call returns a status; a non-zero one becomes a
# `PamgError` carrying the code's name and pamg_last_error(). Handles are freed by finalizers
# (or `close`). Julia arrays passed in are copied by the library. Indices the caller passes
# are 1-based (Julia); the binding converts them where the C side wants 0-based ones.
module PamgHIP

using LinearAlgebra
using SparseArrays

# Exported names never coincide with PartitionedArrays' or LinearAlgebra's (VERDICT r2): the
# PartitionedArrays surface (consistent!, own_values, ghost_values, partition, ...) is extended
# by the package extension with methods of PartitionedArrays' own generic functions, so a solver
# that does `using PartitionedArrays, PamgHIP` calls them unqualified and unambiguously.
export Context, ExchangePlan, DeviceVector, DeviceMatrix, HostCSR, VCycle, ExchangeTask, PamgError,
       download_own, download_ghosts, exchange_begin, residual!, jacobi!, jacobi_residual!, vcycle!, pcg!, set_sweeps!,
       set_perm!, setup_hierarchy, gen_grid, gen_xstar, read_mtx, rcm_order, locality_order, unique_id,
       comm_init!, runtime_versions, hip, World, world_spmv!, world_exchange!, world_dot, world_vcycle!,
       world_pcg!, world_abort!, world_reset!, world_broken, set_tag!

"""
    hip(ctxs, A::PSparseMatrix) / hip(ctxs, x::PVector)

Move PartitionedArrays parts onto the GPU(s); methods live in the PartitionedArrays package
extension (ext/PamgHIPPartitionedArraysExt.jl), loaded when PartitionedArrays is.
"""
function hip end

const libpamg = get(ENV, "PAMG_LIB",
                    normpath(joinpath(@__DIR__, "..", "..", "..", "parallel_amg_amd", "libpamg.so")))

# ------------------------------------------------------------------ errors
const ERRNAMES = Dict{Cint,Symbol}(-1 => :PAMG_E_ARG, -2 => :PAMG_E_HIP, -3 => :PAMG_E_RCCL,
                                   -4 => :PAMG_E_OVERFLOW, -5 => :PAMG_E_SETUP,
                                   -6 => :PAMG_E_STATE, -7 => :PAMG_E_NOMEM)

struct PamgError <: Exception
    code::Cint
    name::Symbol
    msg::String
end
Base.showerror(io::IO, e::PamgError) = print(io, "PamgError(", e.name, "): ", e.msg)

last_error() = unsafe_string(ccall((:pamg_last_error, libpamg), Cstring, ()))
version() = unsafe_string(ccall((:pamg_version, libpamg), Cstring, ()))

function check(rc::Cint)
    rc == 0 && return nothing
    throw(PamgError(rc, get(ERRNAMES, rc, :PAMG_E_UNKNOWN), last_error()))
end

# ------------------------------------------------------------------ context (backend object)
mutable struct Context
    h::Ptr{Cvoid}
    device::Int
    world::Any     # the World this context is a part of (in-process transport), or nothing
end
function Context(device::Integer = 0)
    h = Ref{Ptr{Cvoid}}(C_NULL)
    check(ccall((:pamg_ctx_create, libpamg), Cint, (Cint, Ptr{Ptr{Cvoid}}), device, h))
    ctx = Context(h[], device, nothing)
    finalizer(close, ctx)
end
function Base.close(c::Context)
    c.h == C_NULL && return nothing
    ccall((:pamg_ctx_destroy, libpamg), Cint, (Ptr{Cvoid},), c.h)
    c.h = C_NULL
    nothing
end
sync(c::Context) = check(ccall((:pamg_ctx_sync, libpamg), Cint, (Ptr{Cvoid},), c.h))
"References held on the context (its handle + one per live plan, vector, matrix, hierarchy)."
function refcount(c::Context)
    n = Ref{Cint}(0)
    check(ccall((:pamg_ctx_refcount, libpamg), Cint, (Ptr{Cvoid}, Ptr{Cint}), c.h, n))
    Int(n[])
end
function device_count()
    n = Ref{Cint}(0)
    check(ccall((:pamg_device_count, libpamg), Cint, (Ptr{Cint},), n))
    Int(n[])
end
device_sync(device::Integer) = check(ccall((:pamg_device_sync, libpamg), Cint, (Cint,), device))

"(hip_runtime, hip_built, rccl_runtime, rccl_built) of this process."
function runtime_versions()
    v = [Ref{Cint}(0) for _ in 1:4]
    check(ccall((:pamg_runtime_versions, libpamg), Cint, (Ptr{Cint}, Ptr{Cint}, Ptr{Cint}, Ptr{Cint}),
                v[1], v[2], v[3], v[4]))
    Tuple(Int(r[]) for r in v)
end

# RCCL communicator (the with_mpi backend): rank 0 makes the id, MPI.Bcast! sends the 128
# bytes, every rank calls comm_init!. Load libpamg before anything that brings its own ROCm
# copy; comm_init! refuses an RCCL older than the one libpamg was built against.
function unique_id()
    id = zeros(UInt8, 128)
    check(ccall((:pamg_comm_unique_id, libpamg), Cint, (Ptr{UInt8},), id))
    id
end
comm_init!(ctx::Context, nranks::Integer, rank::Integer, id::Vector{UInt8}) =
    check(ccall((:pamg_comm_init, libpamg), Cint, (Ptr{Cvoid}, Cint, Cint, Ptr{UInt8}),
                ctx.h, nranks, rank, id))
function comm_rank(ctx::Context)
    r, n = Ref{Cint}(0), Ref{Cint}(1)
    check(ccall((:pamg_comm_rank, libpamg), Cint, (Ptr{Cvoid}, Ptr{Cint}, Ptr{Cint}), ctx.h, r, n))
    (Int(r[]), Int(n[]))
end

# ------------------------------------------------------------------ in-process world (with_debug)
"""
    World(nparts; devices = [0])

PartitionedArrays `with_debug` on the device: `nparts` contexts in this process (part p on
`devices[mod1(p, end)]`; parts may share a GPU), registered in one libpamg world, so ghost
exchanges move data by device-to-device copies straight from the sibling parts' vectors
(pamg_comm_init_local). A part's exchange waits for its neighbours' inside the library, so an
operation that exchanges runs for all parts at once: `world_spmv!`, `world_exchange!`,
`world_dot`, `world_vcycle!`, `world_pcg!` (one host thread per part inside libpamg; the
PartitionedArrays extension calls them from its with_debug methods).
"""
mutable struct World
    h::Ptr{Cvoid}
    ctxs::Vector{Context}
end
function World(nparts::Integer; devices::AbstractVector{<:Integer} = [0])
    h = Ref{Ptr{Cvoid}}(C_NULL)
    check(ccall((:pamg_world_create, libpamg), Cint, (Cint, Ptr{Ptr{Cvoid}}), nparts, h))
    w = World(h[], Context[])
    finalizer(close, w)
    for r in 0:nparts-1
        c = Context(devices[mod1(r + 1, length(devices))])
        check(ccall((:pamg_comm_init_local, libpamg), Cint, (Ptr{Cvoid}, Ptr{Cvoid}, Cint), c.h, w.h, r))
        c.world = w
        push!(w.ctxs, c)
    end
    w
end
"Drop the world handle (libpamg keeps the world until its last context is destroyed too)."
function Base.close(w::World)
    w.h == C_NULL && return nothing
    ccall((:pamg_world_destroy, libpamg), Cint, (Ptr{Cvoid},), w.h)
    w.h = C_NULL
    nothing
end
_handles(objs) = Ptr{Cvoid}[o.h for o in objs]
"ys[p] = As[p] xs[p] for every part (the exchanges between siblings included)."
world_spmv!(w::World, ys, As, xs) =
    check(ccall((:pamg_world_spmv, libpamg), Cint, (Ptr{Cvoid}, Ptr{Ptr{Cvoid}}, Ptr{Ptr{Cvoid}}, Ptr{Ptr{Cvoid}}),
                w.h, _handles(As), _handles(xs), _handles(ys)))
"consistent!(x) |> wait for every part: the owners' values into the ghost slots."
world_exchange!(w::World, xs, plans) =
    check(ccall((:pamg_world_exchange, libpamg), Cint, (Ptr{Cvoid}, Ptr{Ptr{Cvoid}}, Ptr{Ptr{Cvoid}}),
                w.h, _handles(plans), _handles(xs)))
"dot over the own entries of every part."
function world_dot(w::World, xs, ys)
    out = Ref{Cdouble}(0.0)
    check(ccall((:pamg_world_dot, libpamg), Cint, (Ptr{Cvoid}, Ptr{Ptr{Cvoid}}, Ptr{Ptr{Cvoid}}, Ptr{Cdouble}),
                w.h, _handles(xs), _handles(ys), out))
    out[]
end
"""
    world_vcycle!(w, xs, Ms, bs; ncycles = 1, hist = true)

ncycles V-cycles on every part's hierarchy; returns the residual history (part 1's = all
parts'), or `nothing` with `hist = false` — then no residual norm (and no all-reduce) is
computed per cycle and stationary runs take the pipelined cycles (the preconditioner's case).
"""
function world_vcycle!(w::World, xs, Ms, bs; ncycles::Integer = 1, hist::Bool = true)
    h = hist ? zeros(Float64, ncycles) : nothing
    check(ccall((:pamg_world_vcycle, libpamg), Cint,
                (Ptr{Cvoid}, Ptr{Ptr{Cvoid}}, Ptr{Ptr{Cvoid}}, Ptr{Ptr{Cvoid}}, Cint, Ptr{Float64}),
                w.h, _handles(Ms), _handles(xs), _handles(bs), ncycles, hist ? h : C_NULL))
    h
end
"Mark the world broken (pamg_world_abort): parts waiting in an exchange fail instead of waiting 300 s."
world_abort!(w::World) = check(ccall((:pamg_world_abort, libpamg), Cint, (Ptr{Cvoid},), w.h))
"Whether the world is broken (a collective failed or was abandoned; pamg_world_state)."
function world_broken(w::World)
    b = Ref{Cint}(0)
    check(ccall((:pamg_world_state, libpamg), Cint, (Ptr{Cvoid}, Ptr{Cint}), w.h, b))
    b[] != 0
end
"Clear a broken world (pamg_world_reset); only when no part is inside a libpamg call."
world_reset!(w::World) = check(ccall((:pamg_world_reset, libpamg), Cint, (Ptr{Cvoid},), w.h))
"PCG with the V-cycle preconditioner on every part; returns (iterations, residual history)."
function world_pcg!(w::World, xs, Ms, bs; rtol::Real = 1e-8, maxit::Integer = 100)
    it = Ref{Cint}(0)
    hist = zeros(Float64, maxit + 1)
    check(ccall((:pamg_world_pcg, libpamg), Cint,
                (Ptr{Cvoid}, Ptr{Ptr{Cvoid}}, Ptr{Ptr{Cvoid}}, Ptr{Ptr{Cvoid}}, Cdouble, Cint, Ptr{Cint}, Ptr{Float64}),
                w.h, _handles(Ms), _handles(xs), _handles(bs), rtol, maxit, it, hist))
    (Int(it[]), hist[1:Int(it[])+1])
end

# ------------------------------------------------------------------ exchange plan (PRange part)
"""
    ExchangePlan(ctx, n_own, n_ghost, nbr_ranks, recv_counts, send_counts, send_idx)

The ghost layout of one part: ghosts occupy slots `n_own+1 : n_own+n_ghost` grouped by
neighbour in `nbr_ranks` order (`recv_counts` each); `send_idx` are the 1-based own indices
sent to each neighbour, concatenated in the same order (`send_counts` each). Ranks are 0-based.
"""
mutable struct ExchangePlan
    h::Ptr{Cvoid}
    ctx::Context
    n_own::Int
    n_ghost::Int
end
function ExchangePlan(ctx::Context, n_own::Integer, n_ghost::Integer, nbr_ranks::AbstractVector{<:Integer},
                      recv_counts::AbstractVector{<:Integer}, send_counts::AbstractVector{<:Integer},
                      send_idx::AbstractVector{<:Integer})
    nb = Int32.(nbr_ranks)
    rc, sc = Int64.(recv_counts), Int64.(send_counts)
    si = Int64.(send_idx) .- 1
    h = Ref{Ptr{Cvoid}}(C_NULL)
    check(ccall((:pamg_plan_create, libpamg), Cint,
                (Ptr{Cvoid}, Int64, Int64, Cint, Ptr{Int32}, Ptr{Int64}, Ptr{Int64}, Ptr{Int64}, Ptr{Ptr{Cvoid}}),
                ctx.h, n_own, n_ghost, length(nb), nb, rc, sc, si, h))
    p = ExchangePlan(h[], ctx, n_own, n_ghost)
    finalizer(close, p)
end
"The plan's index-space identity (pamg_plan_set_tag), the same on every part."
set_tag!(p::ExchangePlan, tag::Integer) =
    check(ccall((:pamg_plan_set_tag, libpamg), Cint, (Ptr{Cvoid}, Int64), p.h, tag))
function Base.close(p::ExchangePlan)
    p.h == C_NULL && return nothing
    ccall((:pamg_plan_destroy, libpamg), Cint, (Ptr{Cvoid},), p.h)
    p.h = C_NULL
    nothing
end

# ------------------------------------------------------------------ vectors (PVector part)
# Not an AbstractVector: its values live on the GPU, and the generic AbstractVector fallbacks
# (show, broadcasting, sum, getindex loops) would copy the whole vector to the host per element.
# Host access is explicit: download_own / download_ghosts / copyto!.
mutable struct DeviceVector
    h::Ptr{Cvoid}
    ctx::Context
    n_own::Int
    n_ghost::Int
end
function DeviceVector(ctx::Context, n_own::Integer, n_ghost::Integer = 0)
    h = Ref{Ptr{Cvoid}}(C_NULL)
    check(ccall((:pamg_vec_create, libpamg), Cint, (Ptr{Cvoid}, Int64, Int64, Ptr{Ptr{Cvoid}}),
                ctx.h, n_own, n_ghost, h))
    v = DeviceVector(h[], ctx, n_own, n_ghost)
    finalizer(close, v)
end
DeviceVector(ctx::Context, own::AbstractVector{<:Real}, n_ghost::Integer = 0) =
    copyto!(DeviceVector(ctx, length(own), n_ghost), own)
function Base.close(v::DeviceVector)
    v.h == C_NULL && return nothing
    ccall((:pamg_vec_destroy, libpamg), Cint, (Ptr{Cvoid},), v.h)
    v.h = C_NULL
    nothing
end
Base.size(v::DeviceVector) = (v.n_own,)
Base.length(v::DeviceVector) = v.n_own
Base.similar(v::DeviceVector) = DeviceVector(v.ctx, v.n_own, v.n_ghost)
Base.show(io::IO, v::DeviceVector) = print(io, "DeviceVector(", v.n_own, " own + ", v.n_ghost, " ghost on GPU ", v.ctx.device, ")")

function Base.copyto!(v::DeviceVector, own::AbstractVector{<:Real})
    length(own) == v.n_own || throw(DimensionMismatch("$(length(own)) values for $(v.n_own) own entries"))
    a = Vector{Float64}(own)
    check(ccall((:pamg_vec_upload, libpamg), Cint, (Ptr{Cvoid}, Ptr{Cvoid}, Ptr{Float64}), v.ctx.h, v.h, a))
    v
end
"The own values, copied to the host."
function download_own(v::DeviceVector)
    out = Vector{Float64}(undef, v.n_own)
    check(ccall((:pamg_vec_download, libpamg), Cint, (Ptr{Cvoid}, Ptr{Cvoid}, Ptr{Float64}), v.ctx.h, v.h, out))
    out
end
"The ghost slots as last exchanged, copied to the host (debugging, tests)."
function download_ghosts(v::DeviceVector)
    out = Vector{Float64}(undef, v.n_ghost)
    check(ccall((:pamg_vec_download_ghosts, libpamg), Cint, (Ptr{Cvoid}, Ptr{Cvoid}, Ptr{Float64}),
                v.ctx.h, v.h, out))
    out
end
function device_pointer(v::DeviceVector)
    p = Ref{Ptr{Float64}}(C_NULL)
    check(ccall((:pamg_vec_device_ptr, libpamg), Cint, (Ptr{Cvoid}, Ptr{Ptr{Float64}}), v.h, p))
    p[]
end
Base.fill!(v::DeviceVector, a::Real) =
    (check(ccall((:pamg_vec_fill, libpamg), Cint, (Ptr{Cvoid}, Ptr{Cvoid}, Cdouble), v.ctx.h, v.h, a)); v)
Base.copy!(dst::DeviceVector, src::DeviceVector) =
    (check(ccall((:pamg_vec_copy, libpamg), Cint, (Ptr{Cvoid}, Ptr{Cvoid}, Ptr{Cvoid}), dst.ctx.h, src.h, dst.h)); dst)
"y = a x + b y (own entries)."
LinearAlgebra.axpby!(a::Real, x::DeviceVector, b::Real, y::DeviceVector) =
    (check(ccall((:pamg_vec_axpby, libpamg), Cint, (Ptr{Cvoid}, Cdouble, Ptr{Cvoid}, Cdouble, Ptr{Cvoid}),
                 y.ctx.h, a, x.h, b, y.h)); y)
LinearAlgebra.axpy!(a::Real, x::DeviceVector, y::DeviceVector) = axpby!(a, x, 1.0, y)
LinearAlgebra.rmul!(y::DeviceVector, b::Real) = axpby!(0.0, y, b, y)
"dot over own entries; with an RCCL communicator the sum over all ranks."
function LinearAlgebra.dot(x::DeviceVector, y::DeviceVector)
    out = Ref{Cdouble}(0.0)
    check(ccall((:pamg_vec_dot, libpamg), Cint, (Ptr{Cvoid}, Ptr{Cvoid}, Ptr{Cvoid}, Ptr{Cdouble}),
                x.ctx.h, x.h, y.h, out))
    out[]
end
function LinearAlgebra.norm(x::DeviceVector)
    out = Ref{Cdouble}(0.0)
    check(ccall((:pamg_vec_nrm2, libpamg), Cint, (Ptr{Cvoid}, Ptr{Cvoid}, Ptr{Cdouble}), x.ctx.h, x.h, out))
    out[]
end

# The device half of PartitionedArrays' consistent!(x) |> wait: exchange_begin enqueues the
# ghost exchange on the context's comm stream and returns at once; wait(t) joins it.
mutable struct ExchangeTask
    x::DeviceVector
    plan::ExchangePlan
    done::Bool
end
function exchange_begin(x::DeviceVector, plan::ExchangePlan)
    check(ccall((:pamg_exchange_begin, libpamg), Cint, (Ptr{Cvoid}, Ptr{Cvoid}, Ptr{Cvoid}),
                x.ctx.h, plan.h, x.h))
    ExchangeTask(x, plan, false)
end
function Base.wait(t::ExchangeTask)
    if !t.done
        check(ccall((:pamg_exchange_end, libpamg), Cint, (Ptr{Cvoid}, Ptr{Cvoid}, Ptr{Cvoid}),
                    t.x.ctx.h, t.plan.h, t.x.h))
        t.done = true
    end
    t.x
end
exchange_ghosts!(x::DeviceVector, plan::ExchangePlan) =
    (check(ccall((:pamg_exchange, libpamg), Cint, (Ptr{Cvoid}, Ptr{Cvoid}, Ptr{Cvoid}), x.ctx.h, plan.h, x.h)); x)

# ------------------------------------------------------------------ matrices (PSparseMatrix part)
mutable struct DeviceMatrix
    h::Ptr{Cvoid}
    ctx::Context
    nrows::Int
    ncols_local::Int
    plan::Union{Nothing,ExchangePlan}
end
"""
    DeviceMatrix(ctx, rowptr, col, val, ncols_local; plan = nothing, index_base = 1,
                 row_perm = nothing, col_perm = nothing)

One part's own rows in CSR with LOCAL column ids (own columns first, then the plan's ghost
slots), each row in ascending global column order (SPEC §S1). Int64 or Int32 columns, 1- or
0-based (`index_base`). The library copies the arrays. `row_perm` / `col_perm` (1-based, one
part): the locality permutation of pamg_mat_upload_perm — device row i is row row_perm[i],
device own column k is own column col_perm[k]; rows keep their storage order (same bits).
"""
function DeviceMatrix(ctx::Context, rowptr::AbstractVector{<:Integer}, col::AbstractVector{<:Integer},
                      val::AbstractVector{<:Real}, ncols_local::Integer;
                      plan::Union{Nothing,ExchangePlan} = nothing, index_base::Integer = 1,
                      row_perm::Union{Nothing,AbstractVector{<:Integer}} = nothing,
                      col_perm::Union{Nothing,AbstractVector{<:Integer}} = nothing)
    rp = Vector{Int64}(rowptr)
    c = eltype(col) == Int32 ? Vector{Int32}(col) : Vector{Int64}(col)
    is64 = eltype(c) == Int64 ? Cint(1) : Cint(0)
    v = Vector{Float64}(val)
    h = Ref{Ptr{Cvoid}}(C_NULL)
    if row_perm === nothing && col_perm === nothing
        check(ccall((:pamg_mat_upload, libpamg), Cint,
                    (Ptr{Cvoid}, Int64, Int64, Ptr{Int64}, Ptr{Cvoid}, Cint, Ptr{Float64}, Cint, Ptr{Cvoid}, Ptr{Ptr{Cvoid}}),
                    ctx.h, length(rp) - 1, ncols_local, rp, c, is64, v, index_base,
                    plan === nothing ? C_NULL : plan.h, h))
    else
        rperm = row_perm === nothing ? Ptr{Int64}(C_NULL) : Int64.(row_perm) .- 1
        cperm = col_perm === nothing ? Ptr{Int64}(C_NULL) : Int64.(col_perm) .- 1
        check(ccall((:pamg_mat_upload_perm, libpamg), Cint,
                    (Ptr{Cvoid}, Int64, Int64, Ptr{Int64}, Ptr{Cvoid}, Cint, Ptr{Float64}, Cint, Ptr{Cvoid},
                     Ptr{Int64}, Ptr{Int64}, Ptr{Ptr{Cvoid}}),
                    ctx.h, length(rp) - 1, ncols_local, rp, c, is64, v, index_base,
                    plan === nothing ? C_NULL : plan.h, rperm, cperm, h))
    end
    A = DeviceMatrix(h[], ctx, length(rp) - 1, ncols_local, plan)
    finalizer(close, A)
end
"A SparseMatrixCSC part (its transpose's CSC arrays are the CSR arrays of the part)."
function DeviceMatrix(ctx::Context, At::SparseMatrixCSC; plan::Union{Nothing,ExchangePlan} = nothing)
    # At = transpose of the part: column j of At is row j of the part
    DeviceMatrix(ctx, At.colptr, At.rowval, At.nzval, size(At, 1); plan = plan, index_base = 1)
end
function Base.close(A::DeviceMatrix)
    A.h == C_NULL && return nothing
    ccall((:pamg_mat_destroy, libpamg), Cint, (Ptr{Cvoid},), A.h)
    A.h = C_NULL
    nothing
end
function info(A::DeviceMatrix)
    nr, nc, nz = Ref{Int64}(0), Ref{Int64}(0), Ref{Int64}(0)
    check(ccall((:pamg_mat_info, libpamg), Cint, (Ptr{Cvoid}, Ptr{Int64}, Ptr{Int64}, Ptr{Int64}), A.h, nr, nc, nz))
    (nrows = nr[], ncols_local = nc[], nnz = nz[])
end
function stream_bytes(A::DeviceMatrix)
    b = Ref{Int64}(0)
    check(ccall((:pamg_mat_stream_bytes, libpamg), Cint, (Ptr{Cvoid}, Ptr{Int64}), A.h, b))
    b[]
end
function layout(A::DeviceMatrix, set::Integer = 0)
    out = zeros(Cint, 10)
    check(ccall((:pamg_mat_layout, libpamg), Cint, (Ptr{Cvoid}, Cint, Ptr{Cint}), A.h, set, out))
    (c24 = out[1] != 0, vd = out[2] != 0, rl8 = out[3] != 0, cd = Int(out[4]), cd_offsets = Int(out[5]),
     tm = out[6] != 0, tm_rs = Int(out[7]), tile_nnz = Int(out[8]), tiles = Int(out[9]), anchored = (out[10] & 1) != 0, per_tile = (out[10] & 2) != 0,
     x_stage = (out[10] & 4) != 0)
end
Base.size(A::DeviceMatrix) = (A.nrows, A.ncols_local)

"mul!(y, A, x): ghost exchange of x (RCCL, overlapped with the interior rows), then y = A x."
LinearAlgebra.mul!(y::DeviceVector, A::DeviceMatrix, x::DeviceVector) =
    (check(ccall((:pamg_spmv, libpamg), Cint, (Ptr{Cvoid}, Ptr{Cvoid}, Ptr{Cvoid}, Ptr{Cvoid}),
                 A.ctx.h, A.h, x.h, y.h)); y)
"r = b - A x; with `norm = true` returns ‖r‖ over all parts instead of r."
function residual!(r::DeviceVector, A::DeviceMatrix, x::DeviceVector, b::DeviceVector; norm::Bool = false)
    nr = Ref{Cdouble}(0.0)
    check(ccall((:pamg_residual, libpamg), Cint,
                (Ptr{Cvoid}, Ptr{Cvoid}, Ptr{Cvoid}, Ptr{Cvoid}, Ptr{Cvoid}, Ptr{Cdouble}),
                A.ctx.h, A.h, x.h, b.h, r.h, norm ? nr : Ptr{Cdouble}(C_NULL)))
    norm ? nr[] : r
end
"nsweeps weighted-Jacobi sweeps x <- x + ω D⁻¹ (b - A x) (tmp: ping-pong buffer)."
jacobi!(x::DeviceVector, A::DeviceMatrix, b::DeviceVector, tmp::DeviceVector, omega::Real, nsweeps::Integer = 1) =
    (check(ccall((:pamg_jacobi, libpamg), Cint,
                 (Ptr{Cvoid}, Ptr{Cvoid}, Ptr{Cvoid}, Ptr{Cvoid}, Ptr{Cvoid}, Cdouble, Cint),
                 A.ctx.h, A.h, x.h, b.h, tmp.h, omega, nsweeps)); x)
"t = x + ω D⁻¹ (b - A x), r = b - A t (one fused pass where the matrix qualifies); returns whether it fused."
function jacobi_residual!(t::DeviceVector, r::DeviceVector, A::DeviceMatrix, x::DeviceVector, b::DeviceVector, omega::Real)
    f = Ref{Cint}(0)
    check(ccall((:pamg_jacobi_residual, libpamg), Cint,
                (Ptr{Cvoid}, Ptr{Cvoid}, Ptr{Cvoid}, Ptr{Cvoid}, Ptr{Cvoid}, Ptr{Cvoid}, Cdouble, Ptr{Cint}),
                A.ctx.h, A.h, x.h, b.h, t.h, r.h, omega, f))
    f[] != 0
end

# ------------------------------------------------------------------ host CSR + setup (SPEC §S4)
mutable struct HostCSR
    h::Ptr{Cvoid}
end
function HostCSR(h::Ptr{Cvoid})
    M = HostCSR(h)
    finalizer(close, M)
end
function HostCSR(nrows::Integer, ncols::Integer, nnz::Integer)
    h = Ref{Ptr{Cvoid}}(C_NULL)
    check(ccall((:pamg_hcsr_create, libpamg), Cint, (Int64, Int64, Int64, Ptr{Ptr{Cvoid}}), nrows, ncols, nnz, h))
    HostCSR(h[])
end
function Base.close(M::HostCSR)
    M.h == C_NULL && return nothing
    ccall((:pamg_hcsr_destroy, libpamg), Cint, (Ptr{Cvoid},), M.h)
    M.h = C_NULL
    nothing
end
function Base.size(M::HostCSR)
    nr, nc, nz = Ref{Int64}(0), Ref{Int64}(0), Ref{Int64}(0)
    check(ccall((:pamg_hcsr_info, libpamg), Cint, (Ptr{Cvoid}, Ptr{Int64}, Ptr{Int64}, Ptr{Int64}), M.h, nr, nc, nz))
    (Int(nr[]), Int(nc[]))
end
"(rowptr, col, val) as Julia arrays wrapping the library's buffers (0-based ids, no copy)."
function arrays(M::HostCSR)
    nr, nc, nz = Ref{Int64}(0), Ref{Int64}(0), Ref{Int64}(0)
    check(ccall((:pamg_hcsr_info, libpamg), Cint, (Ptr{Cvoid}, Ptr{Int64}, Ptr{Int64}, Ptr{Int64}), M.h, nr, nc, nz))
    rp, c, v = Ref{Ptr{Int64}}(C_NULL), Ref{Ptr{Int32}}(C_NULL), Ref{Ptr{Float64}}(C_NULL)
    check(ccall((:pamg_hcsr_data, libpamg), Cint, (Ptr{Cvoid}, Ptr{Ptr{Int64}}, Ptr{Ptr{Int32}}, Ptr{Ptr{Float64}}),
                M.h, rp, c, v))
    (unsafe_wrap(Array, rp[], nr[] + 1), unsafe_wrap(Array, c[], nz[]), unsafe_wrap(Array, v[], nz[]))
end
function DeviceMatrix(ctx::Context, M::HostCSR; plan::Union{Nothing,ExchangePlan} = nothing,
                      row_perm = nothing, col_perm = nothing)
    rp, c, v = arrays(M)
    DeviceMatrix(ctx, rp, c, v, size(M, 2); plan = plan, index_base = 0, row_perm = row_perm, col_perm = col_perm)
end
"A HostCSR holding copies of 0-based CSR arrays (int64 rowptr, global column ids)."
function HostCSR(rowptr::AbstractVector{<:Integer}, col::AbstractVector{<:Integer}, val::AbstractVector{<:Real},
                 ncols::Integer)
    M = HostCSR(length(rowptr) - 1, ncols, rowptr[end])
    rp, c, v = arrays(M)
    rp .= rowptr
    c .= col
    v .= val
    M
end
"Rows `idx` (1-based local row numbers) of M as (rowptr, col, val), 0-based, copied."
function rows(M::HostCSR, idx::AbstractVector{<:Integer})
    rp, c, v = arrays(M)
    lens = Int64[rp[i+1] - rp[i] for i in idx]
    out_rp = zeros(Int64, length(idx) + 1)
    cumsum!(view(out_rp, 2:length(out_rp)), lens)
    oc = Vector{Int32}(undef, out_rp[end])
    ov = Vector{Float64}(undef, out_rp[end])
    for (k, i) in enumerate(idx)
        oc[out_rp[k]+1:out_rp[k+1]] .= view(c, rp[i]+1:rp[i+1])
        ov[out_rp[k]+1:out_rp[k+1]] .= view(v, rp[i]+1:rp[i+1])
    end
    (out_rp, oc, ov)
end

const KINDS = Dict(:poisson2d => 0, :poisson3d => 1, :aniso3d => 2, :elastic3d => 3)
"Rows r0+1:r1 of the SPEC §S2 grid operator (kind ∈ keys(KINDS))."
function gen_grid(kind::Symbol, nx::Integer, ny::Integer, nz::Integer; eps::Real = 1e-3, r0::Integer = 0,
                  r1::Integer = nx * ny * nz * (kind === :elastic3d ? 3 : 1))
    h = Ref{Ptr{Cvoid}}(C_NULL)
    check(ccall((:pamg_gen_grid, libpamg), Cint, (Cint, Int64, Int64, Int64, Cdouble, Int64, Int64, Ptr{Ptr{Cvoid}}),
                KINDS[kind], nx, ny, nz, eps, r0, r1, h))
    HostCSR(h[])
end
function gen_xstar(i0::Integer, n::Integer, seed::Integer = 20240807)
    out = Vector{Float64}(undef, n)
    check(ccall((:pamg_gen_xstar, libpamg), Cint, (Int64, Int64, UInt64, Ptr{Float64}), i0, n, seed, out))
    out
end
"Rows r0+1:r1 (r1 < 0: all) of a Matrix Market file (e.g. SuiteSparse Flan_1565.mtx)."
function read_mtx(path::AbstractString; r0::Integer = 0, r1::Integer = -1)
    n, h = Ref{Int64}(0), Ref{Ptr{Cvoid}}(C_NULL)
    check(ccall((:pamg_read_mtx, libpamg), Cint, (Cstring, Int64, Int64, Ptr{Int64}, Ptr{Ptr{Cvoid}}),
                path, r0, r1, n, h))
    (HostCSR(h[]), Int(n[]))
end
"File rows `rows` (1-based, in that order) of a Matrix Market file, columns in the file numbering."
function read_mtx_rows(path::AbstractString, rows::AbstractVector{<:Integer})
    r = Int64.(rows) .- 1
    n, h = Ref{Int64}(0), Ref{Ptr{Cvoid}}(C_NULL)
    check(ccall((:pamg_read_mtx_rows, libpamg), Cint, (Cstring, Int64, Ptr{Int64}, Ptr{Int64}, Ptr{Ptr{Cvoid}}),
                path, length(r), r, n, h))
    (HostCSR(h[]), Int(n[]))
end
function mtx_row_counts(path::AbstractString)
    n = Ref{Int64}(0)
    check(ccall((:pamg_mtx_row_counts, libpamg), Cint, (Cstring, Ptr{Int64}, Ptr{Int64}), path, n, C_NULL))
    counts = Vector{Int64}(undef, n[])
    check(ccall((:pamg_mtx_row_counts, libpamg), Cint, (Cstring, Ptr{Int64}, Ptr{Int64}), path, n, counts))
    counts
end

"Reverse Cuthill-McKee order (1-based): new row k is old row order[k] (the graph partitioner)."
function rcm_order(A::HostCSR)
    n = size(A)[1]
    order = Vector{Int64}(undef, n)
    check(ccall((:pamg_rcm_order, libpamg), Cint, (Ptr{Cvoid}, Ptr{Int64}), A.h, order))
    order .+ 1
end

"""
    locality_order(A::HostCSR; mode = :auto) -> (order or nothing, span_before, span_after)

Locality order of a square level operator for the device layout (pamg_locality_order):
`:off` identity, `:auto` reverse Cuthill-McKee only where the numbering is scattered, `:on`
always RCM. `order` is 1-based (new row k = old row order[k]); `nothing` means the identity.
"""
function locality_order(A::HostCSR; mode::Symbol = :auto)
    n = size(A)[1]
    order = Vector{Int64}(undef, n)
    applied, before, after = Ref{Cint}(0), Ref{Cdouble}(0.0), Ref{Cdouble}(0.0)
    check(ccall((:pamg_locality_order, libpamg), Cint, (Ptr{Cvoid}, Cint, Ptr{Int64}, Ptr{Cint}, Ptr{Cdouble}, Ptr{Cdouble}),
                A.h, Dict(:off => 0, :auto => 1, :on => 2)[mode], order, applied, before, after))
    (applied[] != 0 ? order .+ 1 : nothing, before[], after[])
end

# ------------------------------------------------------------------ hierarchy / V-cycle
mutable struct VCycle
    h::Ptr{Cvoid}
    ctx::Context
    A::Vector{DeviceMatrix}          # kept alive: the hierarchy references them
    P::Vector{DeviceMatrix}
    R::Vector{DeviceMatrix}
    omega::Vector{Float64}
    ainv::Matrix{Float64}            # coarsest inverse (reused when a tail joins a larger hierarchy)
    ncycles::Int                     # V-cycles per ldiv! (preconditioner use)
end
"""
    VCycle(ctx, A, P, R, omega, ainv; rep_level = length(A) - 1, rep_offsets = nothing, ncycles = 1)

Device hierarchy from per-level device matrices (pamg_hier_create). `ainv` is the coarsest
inverse (n_c × n_c, column-major = a Julia Matrix). Several ranks: levels ≥ rep_level are held
whole on every rank (SPEC §S7); `rep_offsets` (nranks + 1, 0-based row offsets) say which rows
of level rep_level each rank's restriction yields.
"""
function VCycle(ctx::Context, A::Vector{DeviceMatrix}, P::Vector{DeviceMatrix}, R::Vector{DeviceMatrix},
                omega::Vector{Float64}, ainv::Matrix{Float64}; rep_level::Integer = length(A) - 1,
                rep_offsets::Union{Nothing,Vector{Int64}} = nothing, ncycles::Integer = 1)
    L = length(A)
    length(P) == L - 1 && length(R) == L - 1 && length(omega) == L || throw(DimensionMismatch("levels"))
    pa = Ptr{Cvoid}[a.h for a in A]
    pp = Ptr{Cvoid}[[p.h for p in P]; C_NULL]
    pr = Ptr{Cvoid}[[r.h for r in R]; C_NULL]
    h = Ref{Ptr{Cvoid}}(C_NULL)
    check(ccall((:pamg_hier_create, libpamg), Cint,
                (Ptr{Cvoid}, Cint, Ptr{Ptr{Cvoid}}, Ptr{Ptr{Cvoid}}, Ptr{Ptr{Cvoid}}, Ptr{Float64}, Int64,
                 Ptr{Float64}, Cint, Ptr{Int64}, Ptr{Ptr{Cvoid}}),
                ctx.h, L, pa, pp, pr, omega, size(ainv, 1), ainv, rep_level,
                rep_offsets === nothing ? Ptr{Int64}(C_NULL) : rep_offsets, h))
    M = VCycle(h[], ctx, A, P, R, omega, ainv, ncycles)
    finalizer(close, M)
end
function Base.close(M::VCycle)
    M.h == C_NULL && return nothing
    ccall((:pamg_hier_destroy, libpamg), Cint, (Ptr{Cvoid},), M.h)
    M.h = C_NULL
    nothing
end
set_graph!(M::VCycle, enable::Bool) =
    check(ccall((:pamg_hier_set_graph, libpamg), Cint, (Ptr{Cvoid}, Cint), M.h, enable))
set_sweeps!(M::VCycle, nu1::Integer, nu2::Integer) =
    check(ccall((:pamg_hier_set_sweeps, libpamg), Cint, (Ptr{Cvoid}, Cint, Cint), M.h, nu1, nu2))
"Level-0 numbering of a hierarchy uploaded with locality permutations (1-based; nothing = none)."
function set_perm!(M::VCycle, perm::Union{Nothing,AbstractVector{<:Integer}})
    p = perm === nothing ? Int64[] : Int64.(perm) .- 1
    check(ccall((:pamg_hier_set_perm, libpamg), Cint, (Ptr{Cvoid}, Int64, Ptr{Int64}), M.h, length(p),
                isempty(p) ? Ptr{Int64}(C_NULL) : p))
    M
end
function graph_state(M::VCycle)
    e, c, f = Ref{Cint}(0), Ref{Cint}(0), Ref{Cint}(0)
    check(ccall((:pamg_hier_graph_state, libpamg), Cint, (Ptr{Cvoid}, Ptr{Cint}, Ptr{Cint}, Ptr{Cint}), M.h, e, c, f))
    (enabled = e[] != 0, captured = c[] != 0, failed = f[] != 0)
end
"x <- V(x) ncycles times (SPEC §S6); returns the residual norms after each cycle."
function vcycle!(x::DeviceVector, M::VCycle, b::DeviceVector; ncycles::Integer = M.ncycles)
    hist = Vector{Float64}(undef, ncycles)
    check(ccall((:pamg_vcycle, libpamg), Cint,
                (Ptr{Cvoid}, Ptr{Cvoid}, Ptr{Cvoid}, Ptr{Cvoid}, Cint, Ptr{Float64}),
                M.ctx.h, M.h, x.h, b.h, ncycles, hist))
    hist
end
vcycle_async!(x::DeviceVector, M::VCycle, b::DeviceVector, ncycles::Integer) =
    (check(ccall((:pamg_vcycle_async, libpamg), Cint, (Ptr{Cvoid}, Ptr{Cvoid}, Ptr{Cvoid}, Ptr{Cvoid}, Cint),
                 M.ctx.h, M.h, x.h, b.h, ncycles)); x)
"The preconditioner interface (IterativeSolvers / Krylov `Pl = M`): x = M⁻¹ b, i.e. M.ncycles V-cycles from x = 0."
function LinearAlgebra.ldiv!(x::DeviceVector, M::VCycle, b::DeviceVector)
    fill!(x, 0.0)
    check(ccall((:pamg_vcycle, libpamg), Cint,
                (Ptr{Cvoid}, Ptr{Cvoid}, Ptr{Cvoid}, Ptr{Cvoid}, Cint, Ptr{Float64}),
                M.ctx.h, M.h, x.h, b.h, M.ncycles, C_NULL))
    x
end
"CG preconditioned by one V-cycle (SPEC §S8), entirely on the device; returns (iterations, ‖r_k‖ history)."
function pcg!(x::DeviceVector, M::VCycle, b::DeviceVector; rtol::Real = 1e-8, maxit::Integer = 100)
    hist = zeros(maxit + 1)
    it = Ref{Cint}(0)
    check(ccall((:pamg_pcg, libpamg), Cint,
                (Ptr{Cvoid}, Ptr{Cvoid}, Ptr{Cvoid}, Ptr{Cvoid}, Cdouble, Cint, Ptr{Cint}, Ptr{Float64}),
                M.ctx.h, M.h, x.h, b.h, rtol, maxit, it, hist))
    (Int(it[]), hist[1:it[]+1])
end

"""
    setup_hierarchy(ctx, A::HostCSR; theta = 0.02, max_coarse = 1000, max_levels = 20, gpu_products = true,
                    reorder = :auto)

One-part smoothed-aggregation setup (SPEC §S4) through the C-ABI setup entry points — the
sequence parallel_amg_amd/hierarchy.py and tools/pamg_cdriver.c run — then the device
hierarchy, every level but the coarsest uploaded through its locality order (`reorder`, see
`locality_order`; the V-cycle keeps the caller's numbering and bits). Multi-part setups:
`HIPPVCycle(ctxs, A::PSparseMatrix)` in the PartitionedArrays extension.
"""
function setup_hierarchy(ctx::Context, A0::HostCSR; theta::Real = 0.02, max_coarse::Integer = 1000,
                         max_levels::Integer = 20, gpu_products::Bool = true, ncycles::Integer = 1,
                         reorder::Symbol = :auto)
    A, P, R, omega = HostCSR[A0], HostCSR[], HostCSR[], Float64[]
    while true
        rho = Ref{Cdouble}(0.0)
        check(ccall((:pamg_setup_gershgorin, libpamg), Cint, (Ptr{Cvoid}, Int64, Ptr{Cdouble}), A[end].h, 0, rho))
        push!(omega, 4.0 / (3.0 * rho[]))
        n = size(A[end], 1)
        (n <= max_coarse || length(A) >= max_levels) && break
        agg, nagg = Vector{Int32}(undef, n + 1), Ref{Int64}(0)
        check(ccall((:pamg_setup_aggregate, libpamg), Cint, (Ptr{Cvoid}, Int64, Cdouble, Ptr{Int32}, Ptr{Int64}),
                    A[end].h, 0, theta, agg, nagg))
        (nagg[] == 0 || nagg[] >= n) && break
        T = Ref{Ptr{Cvoid}}(C_NULL)
        check(ccall((:pamg_setup_tentative, libpamg), Cint, (Int64, Ptr{Int32}, Int64, Int64, Int64, Ptr{Ptr{Cvoid}}),
                    n, agg, nagg[], 0, nagg[], T))
        Tm = HostCSR(T[])
        Pl, AP, Rl, Ac = Ref{Ptr{Cvoid}}(C_NULL), Ref{Ptr{Cvoid}}(C_NULL), Ref{Ptr{Cvoid}}(C_NULL), Ref{Ptr{Cvoid}}(C_NULL)
        spgemm!(out, X, Y) = gpu_products ?
            check(ccall((:pamg_dev_spgemm, libpamg), Cint,
                        (Ptr{Cvoid}, Ptr{Cvoid}, Int64, Ptr{Cvoid}, Ptr{Int64}, Int64, Ptr{Cvoid}, Ptr{Ptr{Cvoid}}),
                        ctx.h, X.h, 0, Y.h, Ptr{Int64}(C_NULL), 0, C_NULL, out)) :
            check(ccall((:pamg_setup_spgemm, libpamg), Cint,
                        (Ptr{Cvoid}, Int64, Ptr{Cvoid}, Ptr{Int64}, Int64, Ptr{Cvoid}, Ptr{Ptr{Cvoid}}),
                        X.h, 0, Y.h, Ptr{Int64}(C_NULL), 0, C_NULL, out))
        spgemm!(Pl, A[end], Tm)                                   # A T
        Pm = HostCSR(Pl[])
        check(ccall((:pamg_setup_smooth, libpamg), Cint, (Ptr{Cvoid}, Int64, Ptr{Cvoid}, Ptr{Cvoid}, Cdouble),
                    A[end].h, 0, Tm.h, Pm.h, omega[end]))         # P = T - ω D⁻¹ A T
        close(Tm)
        spgemm!(AP, A[end], Pm)
        APm = HostCSR(AP[])
        if gpu_products
            check(ccall((:pamg_dev_transpose, libpamg), Cint, (Ptr{Cvoid}, Ptr{Cvoid}, Int64, Int64, Int64, Ptr{Ptr{Cvoid}}),
                        ctx.h, Pm.h, 0, 0, nagg[], Rl))
        else
            check(ccall((:pamg_setup_transpose, libpamg), Cint, (Ptr{Cvoid}, Int64, Int64, Int64, Ptr{Ptr{Cvoid}}),
                        Pm.h, 0, 0, nagg[], Rl))
        end
        Rm = HostCSR(Rl[])
        spgemm!(Ac, Rm, APm)                                      # R A P
        close(APm)
        push!(P, Pm); push!(R, Rm); push!(A, HostCSR(Ac[]))
    end
    nc = size(A[end], 1)
    ainv = Matrix{Float64}(undef, nc, nc)
    check(ccall((:pamg_setup_cholinv, libpamg), Cint, (Ptr{Cvoid}, Ptr{Float64}), A[end].h, ainv))
    L = length(A)
    perm = Any[l < L ? locality_order(A[l]; mode = reorder)[1] : nothing for l in 1:L]
    dA = [DeviceMatrix(ctx, A[l]; row_perm = perm[l], col_perm = perm[l]) for l in 1:L]
    dP = [DeviceMatrix(ctx, P[l]; row_perm = perm[l], col_perm = perm[l+1]) for l in 1:L-1]
    dR = [DeviceMatrix(ctx, R[l]; row_perm = perm[l+1], col_perm = perm[l]) for l in 1:L-1]
    M = VCycle(ctx, dA, dP, dR, omega, ainv; ncycles = ncycles)
    perm[1] === nothing || set_perm!(M, perm[1])
    M
end

# ------------------------------------------------------------------ setup entry points (multi-part)
# The per-part building blocks of SPEC §S4 with ghost rows, for a distributed setup driven by
# the caller (parallel_amg_amd/hierarchy.py is the Python version of that driver). Row ids are
# global and 0-based, as in the C-ABI.
function gershgorin(A::HostCSR, row0::Integer)
    rho = Ref{Cdouble}(0.0)
    check(ccall((:pamg_setup_gershgorin, libpamg), Cint, (Ptr{Cvoid}, Int64, Ptr{Cdouble}), A.h, row0, rho))
    rho[]
end
function aggregate(A::HostCSR, row0::Integer, theta::Real)
    n = size(A, 1)
    agg, nagg = Vector{Int32}(undef, n + 1), Ref{Int64}(0)
    check(ccall((:pamg_setup_aggregate, libpamg), Cint, (Ptr{Cvoid}, Int64, Cdouble, Ptr{Int32}, Ptr{Int64}),
                A.h, row0, theta, agg, nagg))
    (agg[1:n], Int(nagg[]))
end
function tentative(agg::Vector{Int32}, nagg::Integer, coarse0::Integer, ncols_global::Integer)
    h = Ref{Ptr{Cvoid}}(C_NULL)
    check(ccall((:pamg_setup_tentative, libpamg), Cint, (Int64, Ptr{Int32}, Int64, Int64, Int64, Ptr{Ptr{Cvoid}}),
                length(agg), agg, nagg, coarse0, ncols_global, h))
    HostCSR(h[])
end
"C = X * Y with Y's own rows from y0 and its ghost rows `Yghost` (global ids `ghost_ids`, ascending)."
function spgemm(X::HostCSR, y0::Integer, Yown::HostCSR, ghost_ids::Vector{Int64} = Int64[],
                Yghost::Union{Nothing,HostCSR} = nothing; ctx::Union{Nothing,Context} = nothing)
    h = Ref{Ptr{Cvoid}}(C_NULL)
    yg = Yghost === nothing ? C_NULL : Yghost.h
    if ctx === nothing
        check(ccall((:pamg_setup_spgemm, libpamg), Cint,
                    (Ptr{Cvoid}, Int64, Ptr{Cvoid}, Ptr{Int64}, Int64, Ptr{Cvoid}, Ptr{Ptr{Cvoid}}),
                    X.h, y0, Yown.h, ghost_ids, length(ghost_ids), yg, h))
    else
        check(ccall((:pamg_dev_spgemm, libpamg), Cint,
                    (Ptr{Cvoid}, Ptr{Cvoid}, Int64, Ptr{Cvoid}, Ptr{Int64}, Int64, Ptr{Cvoid}, Ptr{Ptr{Cvoid}}),
                    ctx.h, X.h, y0, Yown.h, ghost_ids, length(ghost_ids), yg, h))
    end
    HostCSR(h[])
end
smooth!(AT::HostCSR, A::HostCSR, row0::Integer, T::HostCSR, omega::Real) =
    (check(ccall((:pamg_setup_smooth, libpamg), Cint, (Ptr{Cvoid}, Int64, Ptr{Cvoid}, Ptr{Cvoid}, Cdouble),
                 A.h, row0, T.h, AT.h, omega)); AT)
function transpose_piece(P::HostCSR, row0::Integer, c0::Integer, c1::Integer; ctx::Union{Nothing,Context} = nothing)
    h = Ref{Ptr{Cvoid}}(C_NULL)
    if ctx === nothing
        check(ccall((:pamg_setup_transpose, libpamg), Cint, (Ptr{Cvoid}, Int64, Int64, Int64, Ptr{Ptr{Cvoid}}),
                    P.h, row0, c0, c1, h))
    else
        check(ccall((:pamg_dev_transpose, libpamg), Cint, (Ptr{Cvoid}, Ptr{Cvoid}, Int64, Int64, Int64, Ptr{Ptr{Cvoid}}),
                    ctx.h, P.h, row0, c0, c1, h))
    end
    HostCSR(h[])
end
function hstack_rows(pieces::Vector{HostCSR})
    h = Ref{Ptr{Cvoid}}(C_NULL)
    ps = Ptr{Cvoid}[p.h for p in pieces]
    check(ccall((:pamg_setup_hstack_rows, libpamg), Cint, (Cint, Ptr{Ptr{Cvoid}}, Ptr{Ptr{Cvoid}}), length(ps), ps, h))
    HostCSR(h[])
end
function cholinv(A::HostCSR)
    n = size(A, 1)
    ainv = Matrix{Float64}(undef, n, n)
    check(ccall((:pamg_setup_cholinv, libpamg), Cint, (Ptr{Cvoid}, Ptr{Float64}), A.h, ainv))
    ainv
end

# ------------------------------------------------------------------ profiling / micro-benchmarks
function vec_size(v::DeviceVector)
    o, g = Ref{Int64}(0), Ref{Int64}(0)
    check(ccall((:pamg_vec_size, libpamg), Cint, (Ptr{Cvoid}, Ptr{Int64}, Ptr{Int64}), v.h, o, g))
    (Int(o[]), Int(g[]))
end
"ms per (level, op) of `ncycles` eagerly launched V-cycles (HIP events; columns: jacobi_pre, residual, restrict, prolong, jacobi_post, coarse)."
function profile(x::DeviceVector, M::VCycle, b::DeviceVector, ncycles::Integer)
    check(ccall((:pamg_hier_profile, libpamg), Cint, (Ptr{Cvoid}, Cint), M.h, 1))
    try
        vcycle_async!(x, M, b, ncycles)
        out = zeros(6 * length(M.A))
        check(ccall((:pamg_hier_profile_read, libpamg), Cint, (Ptr{Cvoid}, Ptr{Float64}), M.h, out))
        permutedims(reshape(out, 6, length(M.A)))
    finally
        check(ccall((:pamg_hier_profile, libpamg), Cint, (Ptr{Cvoid}, Cint), M.h, 0))
    end
end
"Average ms of `reps` launches of one row operation (0 SpMV, 1 residual, 2 Jacobi, 3 prolongate-add)."
function bench_rowop(A::DeviceMatrix, op::Integer, x::DeviceVector, b::Union{Nothing,DeviceVector},
                     y::DeviceVector; omega::Real = 0.0, reps::Integer = 20)
    ms = Ref{Cdouble}(0.0)
    check(ccall((:pamg_bench_rowop, libpamg), Cint,
                (Ptr{Cvoid}, Ptr{Cvoid}, Cint, Ptr{Cvoid}, Ptr{Cvoid}, Ptr{Cvoid}, Cdouble, Cint, Ptr{Cdouble}),
                A.ctx.h, A.h, op, x.h, b === nothing ? C_NULL : b.h, y.h, omega, reps, ms))
    ms[]
end

"Average ms of `reps` launches of the cross-cycle pipeline's level-0 chain kernel (x is overwritten)."
function bench_chain(x::DeviceVector, M::VCycle, b::DeviceVector; reps::Integer = 10)
    ms = Ref{Cdouble}(0.0)
    check(ccall((:pamg_hier_bench_chain, libpamg), Cint, (Ptr{Cvoid}, Ptr{Cvoid}, Ptr{Cvoid}, Cint, Ptr{Cdouble}),
                M.h, x.h, b.h, reps, ms))
    ms[]
end

# ------------------------------------------------------------------ knobs
set_option!(key::AbstractString, value::Integer) =
    check(ccall((:pamg_set_option, libpamg), Cint, (Cstring, Int64), key, value))
function get_option(key::AbstractString)
    v = Ref{Int64}(0)
    check(ccall((:pamg_get_option, libpamg), Cint, (Cstring, Ptr{Int64}), key, v))
    v[]
end

end # module
