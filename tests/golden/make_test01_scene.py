"""Extract the *scene data* of the reference's tests/test01/test01.c into test01_scene.json.

Run here (where /root/reference exists):  python tests/golden/make_test01_scene.py
The JSON holds numbers only — object vertices/triangles with their material, material diffuse
colour / diffuse_reflect / emit, the point light, the camera and the constant background — i.e.
the inputs of BASELINE config C1 (textures stripped for the C1 plumbing golden).
For the textured variant it also records, as typed parameter maps, every createImage /
createTexture / createMaterial call (with the material's pushed shader-node lists) and the
objects' orco coordinates.  The texture files the images name are the reference's own test data
(tests/test01/tex.*): the TGA and HDR ones are copied to tests/golden/tex01/ (the reference as built
here reads only those two formats).  The GPU box never needs the reference tree.
"""
import json
import os
import re
import sys

SRC = "/root/reference/tests/test01/test01.c"
OUT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "test01_scene.json")

CALL = re.compile(r"yafaray_(\w+)\(yi(?:,\s*(.*))?\);")


def parse_args(s):
    if not s:
        return []
    out = []
    for tok in re.findall(r'"[^"]*"|[^,]+', s):
        tok = tok.strip()
        if tok.startswith('"'):
            out.append(tok[1:-1])
        elif tok.startswith("YAFARAY_BOOL_"):
            out.append(tok.endswith("TRUE"))
        else:
            try:
                out.append(float(tok))
            except ValueError:
                out.append(tok)
    return out


def main():
    if not os.path.exists(SRC):
        sys.exit("reference tree absent; the committed test01_scene.json is used as is")
    params, in_list = {}, False
    typed, nodes = {}, []
    images, textures, materials_full = [], [], []
    kinds = {"paramsSetString": "s", "paramsSetFloat": "f", "paramsSetInt": "i", "paramsSetBool": "b",
             "paramsSetVector": "v", "paramsSetColor": "c"}
    materials, objects, lights = [], [], []
    camera, background, cur_obj, cur_mat = None, None, None, None
    for line in open(SRC):
        m = CALL.search(line)
        if not m:
            continue
        fn, args = m.group(1), parse_args(m.group(2))
        if fn == "paramsClearAll":
            params, in_list = {}, False
            typed, nodes = {}, []
        elif fn == "paramsPushList":
            in_list = True
            nodes.append({})
        elif fn == "paramsEndList":
            in_list = False
        elif fn.startswith("paramsSet"):
            val = args[1:] if len(args) > 2 else args[1]
            tv = [kinds[fn], val]
            if in_list:
                nodes[-1][args[0]] = tv
            else:
                params[args[0]] = val
                typed[args[0]] = tv
        elif fn == "createImage":
            images.append({"name": args[0], "params": typed})
        elif fn == "createTexture":
            textures.append({"name": args[0], "params": typed})
        elif fn == "createMaterial":
            materials_full.append({"name": args[0], "params": typed, "nodes": nodes})
            col = params.get("color", [0.8, 0.8, 0.8, 1.0])
            materials.append({"name": args[0], "color": [float(c) for c in col[:3]],
                              "diffuse_reflect": float(params.get("diffuse_reflect", 1.0)),
                              "emit": float(params.get("emit", 0.0))})
        elif fn == "createLight":
            assert params["type"] == "pointlight"
            lights.append({"name": args[0], "color": [float(c) for c in params["color"][:3]],
                           "power": float(params["power"]), "from": [float(c) for c in params["from"]]})
        elif fn == "createObject":
            cur_obj = {"name": args[0], "verts": [], "orco": [], "tris": [], "material": None}
            objects.append(cur_obj)
        elif fn in ("addVertex", "addVertexWithOrco"):
            cur_obj["verts"].append([float(a) for a in args[:3]])
            if fn == "addVertexWithOrco":
                cur_obj["orco"].append([float(a) for a in args[3:6]])
        elif fn == "setCurrentMaterial":
            cur_mat = args[0]
        elif fn == "addTriangle":
            assert cur_obj["material"] in (None, cur_mat), "one material per object expected"
            cur_obj["material"] = cur_mat
            cur_obj["tris"].append([int(a) for a in args[:3]])
        elif fn == "createCamera":
            camera = {"from": [float(c) for c in params["from"]], "to": [float(c) for c in params["to"]],
                      "up": [float(c) for c in params["up"]], "focal": float(params["focal"]),
                      "resx": int(params["resx"]), "resy": int(params["resy"])}
        elif fn == "createBackground":
            background = {"color": [float(c) for c in params["color"][:3]], "power": float(params["power"])}
    d = {"source": "reference tests/test01/test01.c (scene data; 'materials' has textures stripped, "
                   "'materials_full' / 'images' / 'textures' keep the typed parameter maps)",
         "materials": materials, "objects": objects, "lights": lights, "camera": camera, "background": background,
         "materials_full": materials_full, "images": images, "textures": textures}
    import shutil
    tex_dir = os.path.join(os.path.dirname(OUT), "tex01")
    os.makedirs(tex_dir, exist_ok=True)
    for ext in ("tga", "hdr"):
        shutil.copyfile(os.path.join(os.path.dirname(SRC), "tex." + ext), os.path.join(tex_dir, "tex." + ext))
    with open(OUT, "w") as f:
        json.dump(d, f, indent=0)
    print("wrote", OUT, len(objects), "objects", sum(len(o["tris"]) for o in objects), "triangles")


if __name__ == "__main__":
    main()
