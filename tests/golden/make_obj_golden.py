"""Golden vectors for the OBJ import restatement (raytracing_gpu_amd/csrc/rt_obj.cpp).

The reference imports meshes with assimp (Importer::ReadFile(path, aiProcess_Triangulate |
aiProcess_GenNormals), triangle_mesh.h:129-143) and walks the node tree in processNode order
(:115-126).  No assimp library is installed here, but this container's Qt3D scene-import plugin
(/opt/conda/plugins/sceneparsers/libassimpsceneimport.so) embeds assimp v3.3 and exports its C API;
this script imports each OBJ through it (aiImportFile, flags 0x8 | 0x20) in a child process (the
plugin brings an older libstdc++) and stores, per aiMesh in processNode order: positions,
normals, uv (first channel, x/y), face index lists (-1 padded) and the material index.

Outputs (committed):
  obj/case1.npz, obj/case2.npz  -- the synthetic cases in obj/ (written by hand for this test)
  door_assimp.npz               -- assets/door/door.obj of the reference (config C4), if present

Run in this container only:  python tests/golden/make_obj_golden.py
The reference used assimp 5.x; this pins the restatement against an actual assimp (v3.3).
"""
from __future__ import annotations

import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
PLUGIN = "/opt/conda/plugins/sceneparsers/libassimpsceneimport.so"
DOOR = "/root/reference/assets/door/door.obj"

CHILD = r'''
import ctypes, sys
import numpy as np
from ctypes import c_uint, c_float, c_void_p, c_size_t, c_char, POINTER, Structure
L = ctypes.CDLL(sys.argv[1])
class aiString(Structure): _fields_ = [("length", c_size_t), ("data", c_char * 1024)]
class aiVector3D(Structure): _fields_ = [("x", c_float), ("y", c_float), ("z", c_float)]
class aiFace(Structure): _fields_ = [("mNumIndices", c_uint), ("mIndices", POINTER(c_uint))]
class aiMesh(Structure):
    _fields_ = [("mPrimitiveTypes", c_uint), ("mNumVertices", c_uint), ("mNumFaces", c_uint),
                ("mVertices", POINTER(aiVector3D)), ("mNormals", POINTER(aiVector3D)),
                ("mTangents", POINTER(aiVector3D)), ("mBitangents", POINTER(aiVector3D)),
                ("mColors", c_void_p * 8), ("mTextureCoords", POINTER(aiVector3D) * 8),
                ("mNumUVComponents", c_uint * 8), ("mFaces", POINTER(aiFace)), ("mNumBones", c_uint),
                ("mBones", c_void_p), ("mMaterialIndex", c_uint), ("mName", aiString)]
class aiNode(Structure): pass
aiNode._fields_ = [("mName", aiString), ("mTransformation", c_float * 16), ("mParent", POINTER(aiNode)),
                   ("mNumChildren", c_uint), ("mChildren", POINTER(POINTER(aiNode))), ("mNumMeshes", c_uint),
                   ("mMeshes", POINTER(c_uint))]
class aiScene(Structure):
    _fields_ = [("mFlags", c_uint), ("mRootNode", POINTER(aiNode)), ("mNumMeshes", c_uint),
                ("mMeshes", POINTER(POINTER(aiMesh))), ("mNumMaterials", c_uint), ("mMaterials", c_void_p)]
L.aiImportFile.restype = POINTER(aiScene)
L.aiImportFile.argtypes = [ctypes.c_char_p, c_uint]
L.aiGetVersionMajor.restype = c_uint
L.aiGetVersionMinor.restype = c_uint
sc = L.aiImportFile(sys.argv[2].encode(), 0x8 | 0x20)
if not sc:
    raise SystemExit("assimp failed to import " + sys.argv[2])
s = sc.contents
out = {"version": np.array([L.aiGetVersionMajor(), L.aiGetVersionMinor()], np.int32)}
k = 0
def node(n):
    global k
    n = n.contents
    for i in range(n.mNumMeshes):
        m = s.mMeshes[n.mMeshes[i]].contents
        nv = m.mNumVertices
        out[f"v{k}"] = np.array([(m.mVertices[j].x, m.mVertices[j].y, m.mVertices[j].z) for j in range(nv)], np.float32).reshape(-1, 3)
        out[f"n{k}"] = (np.array([(m.mNormals[j].x, m.mNormals[j].y, m.mNormals[j].z) for j in range(nv)], np.float32)
                        if m.mNormals else np.zeros((nv, 3), np.float32)).reshape(-1, 3)
        out[f"uv{k}"] = (np.array([(m.mTextureCoords[0][j].x, m.mTextureCoords[0][j].y) for j in range(nv)], np.float32)
                         if m.mTextureCoords[0] else np.zeros((nv, 2), np.float32)).reshape(-1, 2)
        faces = [[m.mFaces[f].mIndices[j] for j in range(m.mFaces[f].mNumIndices)] for f in range(m.mNumFaces)]
        w = max([len(f) for f in faces] + [1])
        out[f"f{k}"] = np.array([f + [-1] * (w - len(f)) for f in faces], np.int64).reshape(-1, w)
        out[f"mat{k}"] = np.array([m.mMaterialIndex], np.int32)
        k += 1
    for i in range(n.mNumChildren):
        node(n.mChildren[i])
node(s.mRootNode)
out["n_meshes"] = np.array([k], np.int32)
np.savez_compressed(sys.argv[3], **out)
L.aiReleaseImport(sc)
'''


def run(obj: str, out: str) -> None:
    subprocess.run([sys.executable, "-c", CHILD, PLUGIN, obj, out], check=True)
    print("wrote", out)


def main() -> None:
    if not os.path.exists(PLUGIN):
        raise SystemExit(f"{PLUGIN} not found: the golden OBJ vectors can only be regenerated where it exists")
    for case in ("case1", "case2"):
        run(os.path.join(HERE, "obj", case + ".obj"), os.path.join(HERE, "obj", case + ".npz"))
    if os.path.exists(DOOR):
        run(DOOR, os.path.join(HERE, "door_assimp.npz"))


if __name__ == "__main__":
    main()
