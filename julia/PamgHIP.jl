# PamgHIP.jl — the Julia-side binding of libpamg (include/pamg.h) a PartitionedArrays-based
# AMG code would use. NOT runnable in this image (no Julia, no PartitionedArrays.jl, no
# network); the tested contract is the C-ABI itself (tests/test_abi.py) and its Python
# binding (parallel_amg_amd/_lib.py). See INTEGRATION.md.
module PamgHIP

using LinearAlgebra

const libpamg = joinpath(@__DIR__, "..", "parallel_amg_amd", "libpamg.so")

struct PamgError <: Exception
    code::Cint
    msg::String
end

function check(rc::Cint)
    rc == 0 && return nothing
    msg = unsafe_string(ccall((:pamg_last_error, libpamg), Cstring, ()))
    throw(PamgError(rc, msg))
end

mutable struct Context
    h::Ptr{Cvoid}
end
function Context(device::Integer = 0)
    h = Ref{Ptr{Cvoid}}(C_NULL)
    check(ccall((:pamg_ctx_create, libpamg), Cint, (Cint, Ptr{Ptr{Cvoid}}), device, h))
    ctx = Context(h[])
    finalizer(c -> ccall((:pamg_ctx_destroy, libpamg), Cint, (Ptr{Cvoid},), c.h), ctx)
end

# RCCL communicator: rank 0 makes the id, MPI.Bcast! sends it, every rank calls comm_init!.
function unique_id()
    id = zeros(UInt8, 128)
    check(ccall((:pamg_comm_unique_id, libpamg), Cint, (Ptr{UInt8},), id))
    id
end
comm_init!(ctx::Context, nranks, rank, id::Vector{UInt8}) =
    check(ccall((:pamg_comm_init, libpamg), Cint, (Ptr{Cvoid}, Cint, Cint, Ptr{UInt8}),
                ctx.h, nranks, rank, id))

# Device PVector part: own values then ghost slots.
mutable struct DeviceVector
    ctx::Context
    h::Ptr{Cvoid}
    n_own::Int
end
function DeviceVector(ctx::Context, n_own::Integer, n_ghost::Integer = 0)
    h = Ref{Ptr{Cvoid}}(C_NULL)
    check(ccall((:pamg_vec_create, libpamg), Cint, (Ptr{Cvoid}, Int64, Int64, Ptr{Ptr{Cvoid}}),
                ctx.h, n_own, n_ghost, h))
    v = DeviceVector(ctx, h[], n_own)
    finalizer(x -> ccall((:pamg_vec_destroy, libpamg), Cint, (Ptr{Cvoid},), x.h), v)
end
Base.copyto!(v::DeviceVector, own::Vector{Float64}) =
    (check(ccall((:pamg_vec_upload, libpamg), Cint, (Ptr{Cvoid}, Ptr{Cvoid}, Ptr{Float64}),
                 v.ctx.h, v.h, own)); v)
function own_values(v::DeviceVector)
    out = Vector{Float64}(undef, v.n_own)
    check(ccall((:pamg_vec_download, libpamg), Cint, (Ptr{Cvoid}, Ptr{Cvoid}, Ptr{Float64}),
                v.ctx.h, v.h, out))
    out
end

# Device PSparseMatrix part from the own rows of a SparseMatrixCSC-derived CSR (1-based, Int64
# indices are accepted directly: index_base = 1, col_is_64 = 1).
mutable struct DeviceMatrix
    ctx::Context
    h::Ptr{Cvoid}
end
function DeviceMatrix(ctx::Context, rowptr::Vector{Int64}, col::Vector{Int64}, val::Vector{Float64},
                      ncols_local::Integer, plan::Ptr{Cvoid} = C_NULL)
    h = Ref{Ptr{Cvoid}}(C_NULL)
    check(ccall((:pamg_mat_upload, libpamg), Cint,
                (Ptr{Cvoid}, Int64, Int64, Ptr{Int64}, Ptr{Cvoid}, Cint, Ptr{Float64}, Cint, Ptr{Cvoid}, Ptr{Ptr{Cvoid}}),
                ctx.h, length(rowptr) - 1, ncols_local, rowptr, col, 1, val, 1, plan, h))
    A = DeviceMatrix(ctx, h[])
    finalizer(m -> ccall((:pamg_mat_destroy, libpamg), Cint, (Ptr{Cvoid},), m.h), A)
end

# mul!(y, A, x): ghost exchange of x (RCCL, overlapped with interior rows), then y = A x.
LinearAlgebra.mul!(y::DeviceVector, A::DeviceMatrix, x::DeviceVector) =
    (check(ccall((:pamg_spmv, libpamg), Cint, (Ptr{Cvoid}, Ptr{Cvoid}, Ptr{Cvoid}, Ptr{Cvoid}),
                 A.ctx.h, A.h, x.h, y.h)); y)

# V-cycle preconditioner: ldiv!(x, M, b) runs ncycles V-cycles from x (SPEC §S6).
struct VCycle
    ctx::Context
    h::Ptr{Cvoid}
    ncycles::Int
end
LinearAlgebra.ldiv!(x::DeviceVector, M::VCycle, b::DeviceVector) =
    (check(ccall((:pamg_vcycle, libpamg), Cint,
                 (Ptr{Cvoid}, Ptr{Cvoid}, Ptr{Cvoid}, Ptr{Cvoid}, Cint, Ptr{Float64}),
                 M.ctx.h, M.h, x.h, b.h, M.ncycles, C_NULL)); x)

end # module
